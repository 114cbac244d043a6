"""Where this image keeps the react@18.3.1 / react-dom@18.3.1 UMD builds.

There is no npm registry here; an installed Python package (dash) vendors the
exact React builds package.json pins, development and production (.min.js).
The real-React spec tier (tests/test_js_real_react.py) runs on the first, the
bench's real-React mount / re-render figure (bench/driver.js) on the second.
"""
from __future__ import annotations

import os
from typing import Optional

DEV_BUILDS = ("react@18.3.1.js", "react-dom@18.3.1.js")
PROD_BUILDS = ("react@18.3.1.min.js", "react-dom@18.3.1.min.js")


def umd_dir(builds=DEV_BUILDS) -> Optional[str]:
    """The directory holding `builds`, or None when no installed package vendors them."""
    try:
        import dash  # noqa: PLC0415 — vendors React's UMD builds under dash/deps
    except Exception:  # noqa: BLE001
        return None
    d = os.path.join(os.path.dirname(dash.__file__), "deps")
    return d if all(os.path.exists(os.path.join(d, b)) for b in builds) else None
