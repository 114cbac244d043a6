#!/usr/bin/env python3
"""Run the amdgpu-exporter's HTTP serving under host AddressSanitizer + UBSan (no GPU needed).

    python tools/asan_exporter.py [--build-dir /tmp/asan]

Builds the daemon with `-fsanitize=address,undefined -fno-gpu-sanitize` (host code only; the GPU side is not
instrumented), starts it in --sysfs-only mode and drives it with 300 random payloads, a 20 kB request line, 50
slow-loris peers that reach their deadline, and 50 scrapes, then SIGTERM. It fails on any sanitizer report,
a non-zero exit or a leak at exit.
"""
import argparse
import os
import random
import signal
import socket
import subprocess
import sys
import time
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "headlamp_intel_gpu_plugin_amd", "ops", "csrc")


def build(out_dir):
    os.makedirs(out_dir, exist_ok=True)
    exe = os.path.join(out_dir, "amdgpu-exporter-asan")
    hipcc = "/opt/rocm/bin/hipcc"
    cmd = [hipcc, "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-gpu-sanitize", "-I", CSRC,
           "--offload-arch=gfx950", os.path.join(CSRC, "amdgpu_exporter.cpp"), "-o", exe, "-L/opt/rocm/lib",
           "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"]
    subprocess.run(cmd, check=True, timeout=600)
    return exe


def drive(exe):
    env = {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1", "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1",
           "PATH": "/usr/bin:/bin"}
    p = subprocess.Popen([exe, "--port", "0", "--bind", "127.0.0.1", "--hostname", "asan", "--sysfs-only"],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
    line = p.stdout.readline()
    port = int(line.split("127.0.0.1:")[1].split()[0])
    rnd = random.Random(3)
    payloads = [b"", b"\r\n\r\n", b"GET\r\n\r\n", b"GET / HTTP/1.1", b"GET /" + b"a" * 20000 + b" HTTP/1.1\r\n\r\n"]
    payloads += [bytes(rnd.getrandbits(8) for _ in range(rnd.randint(1, 5000))) for _ in range(300)]
    slow = [socket.create_connection(("127.0.0.1", port)) for _ in range(50)]
    for s in slow:
        s.sendall(b"G")
    for d in payloads:
        with socket.create_connection(("127.0.0.1", port), timeout=5) as s:
            try:
                s.sendall(d)
                s.shutdown(socket.SHUT_WR)
                s.recv(65536)
            except OSError:
                pass
    for _ in range(50):
        with urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5) as r:
            r.read()
    time.sleep(3.5)  # the slow peers reach their request deadline
    for s in slow:
        s.close()
    with urllib.request.urlopen(f"http://127.0.0.1:{port}/healthz", timeout=5) as r:
        assert r.read() == b"ok\n"
    p.send_signal(signal.SIGTERM)
    rc = p.wait(30)
    err = p.stderr.read()
    ok = rc == 0 and "ERROR: AddressSanitizer" not in err and "runtime error" not in err and "LeakSanitizer" not in err
    return ok, rc, err


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build-dir", default="/tmp/asan")
    a = ap.parse_args()
    ok, rc, err = drive(build(a.build_dir))
    print(f"exit {rc}; sanitizer clean: {ok}")
    if not ok:
        print(err[-5000:])
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
