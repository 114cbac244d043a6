"""The hand-written .d.ts files type the plain-JS modules next to them (src/**); no TypeScript compiler is
available offline, so this pins the part a drift would break first: every value a module exports is declared in
its .d.ts, and every value the .d.ts declares is exported (types and interfaces are .d.ts-only)."""
import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PAIRS = sorted(p[:-5] for p in glob.glob(os.path.join(ROOT, "src", "**", "*.d.ts"), recursive=True)
               if os.path.exists(p[:-5] + ".js"))

DECL = re.compile(r"^export (?:declare )?(?:async )?(?:function\*?|const|let|var|class) ([A-Za-z_$][\w$]*)", re.M)
LIST = re.compile(r"^export \{([^}]*)\}(?: from '[^']+')?;", re.M)
DESTRUCT = re.compile(r"^export (?:const|let|var) \{([^}]*)\}", re.M)


def exported(text):
    names = set(DECL.findall(text))
    for body in LIST.findall(text) + DESTRUCT.findall(text):
        for part in body.split(","):
            part = part.strip()
            if part:
                names.add(re.split(r"\s+as\s+|\s*:\s*", part)[-1].strip())
    return names


def test_pairs_found():
    rel = [os.path.relpath(p, ROOT) for p in PAIRS]
    assert {"src/api/providerCore", "src/plugin", "src/view/ir", "src/view/react", "src/view/settingsPage"} <= set(rel)


@pytest.mark.parametrize("base", PAIRS, ids=lambda p: os.path.relpath(p, ROOT))
def test_values_match(base):
    js = exported(open(base + ".js").read())
    dts = exported(open(base + ".d.ts").read())
    assert js - dts == set(), f"exported by {os.path.relpath(base, ROOT)}.js but not declared"
    assert dts - js == set(), f"declared in {os.path.relpath(base, ROOT)}.d.ts but not exported"
