"""Drive the Node.js benchmark driver (bench/driver.js --serve) from Python."""
from __future__ import annotations

import json
import os
import shutil
import subprocess
from typing import Dict, Optional

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def node_binary() -> str:
    n = shutil.which("node") or shutil.which("nodejs")
    if not n:
        raise RuntimeError("node is required to run the plugin's data layer")
    return n


class Driver:
    """A long-lived ``bench/driver.js --serve`` process speaking JSON lines."""

    def __init__(self, url: str, node_flags=(), env: Optional[Dict[str, str]] = None):
        # HEADLAMP_AMD_NODE_FLAGS: extra node flags for diagnostics, e.g. "--cpu-prof --cpu-prof-dir=/tmp/p"
        # (node 12 refuses --cpu-prof in NODE_OPTIONS). `node_flags` / `env`: the opt-in render comparison runs the
        # driver with --disallow-code-generation-from-strings and a minimal environment (tools/render_compare.py).
        flags = list(node_flags) + os.environ.get("HEADLAMP_AMD_NODE_FLAGS", "").split()
        self.proc = subprocess.Popen([node_binary(), *flags, os.path.join(ROOT, "bench", "driver.js"), "--serve", "--url", url],
                                     cwd=ROOT, stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                     text=True, bufsize=1, env=env)

    def call(self, cmd: str, schedule: str = "amd", n: int = 1, timeout: Optional[float] = None, **extra) -> Dict:
        assert self.proc.stdin and self.proc.stdout
        self.proc.stdin.write(json.dumps(dict({"cmd": cmd, "schedule": schedule, "n": n}, **extra)) + "\n")
        self.proc.stdin.flush()
        line = self.proc.stdout.readline()
        if not line:
            err = self.proc.stderr.read() if self.proc.stderr else ""
            raise RuntimeError(f"driver exited: {err[-2000:]}")
        out = json.loads(line)
        if "error" in out:
            raise RuntimeError(out["error"])
        return out

    def close(self) -> None:
        if self.proc.poll() is None:
            try:
                self.proc.stdin.write(json.dumps({"cmd": "quit"}) + "\n")
                self.proc.stdin.flush()
                self.proc.wait(5)
            except (OSError, subprocess.TimeoutExpired):
                self.proc.kill()
                self.proc.wait(5)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
