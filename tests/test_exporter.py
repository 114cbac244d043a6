"""Native amdgpu-exporter daemon (ops/csrc/amdgpu_exporter.cpp).

CPU tests run the binary with no GPU (it must still answer, with no GPU series);
the GPU test checks real MI355X series and the single-device relabelling mode.
"""
import os
import re
import shutil
import signal
import subprocess
import time
import urllib.error
import urllib.request

import pytest

from headlamp_intel_gpu_plugin_amd.ops import build as native_build
from headlamp_intel_gpu_plugin_amd.ops.probe import parse_exposition

HAS_HIPCC = bool(shutil.which("hipcc") or os.path.exists("/opt/rocm/bin/hipcc"))
pytestmark = pytest.mark.skipif(not HAS_HIPCC, reason="hipcc not available")


@pytest.fixture(scope="module")
def exe():
    return native_build.build(["amdgpu-exporter"])["amdgpu-exporter"]


@pytest.fixture()
def server(exe):
    p = subprocess.Popen([exe, "--port", "0", "--bind", "127.0.0.1", "--hostname", "mi355x-test"],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    line = p.stdout.readline()
    assert "listening on" in line, line + p.stderr.read()
    port = int(line.split("127.0.0.1:")[1].split()[0])
    yield p, f"http://127.0.0.1:{port}"
    if p.poll() is None:
        p.send_signal(signal.SIGTERM)
        p.wait(10)


def test_once_prints_help_and_types(exe):
    r = subprocess.run([exe, "--once", "--hostname", "n0"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0
    assert "# TYPE gpu_power_usage gauge" in r.stdout
    assert "# HELP gpu_xgmi_link_hops" in r.stdout


def test_rejects_bad_arguments(exe):
    assert subprocess.run([exe, "--bogus"], capture_output=True, timeout=30).returncode == 2
    assert subprocess.run([exe, "--port", "70000"], capture_output=True, timeout=30).returncode == 2


def test_http_endpoints(server):
    _, url = server
    with urllib.request.urlopen(url + "/healthz", timeout=10) as r:
        assert r.status == 200 and r.read() == b"ok\n"
    with urllib.request.urlopen(url + "/metrics", timeout=10) as r:
        assert r.headers["Content-Type"].startswith("text/plain")
        body = r.read().decode()
    assert "# TYPE gpu_total_vram gauge" in body
    for name, labels, _ in parse_exposition(body):
        assert labels["hostname"] == "mi355x-test"
    with pytest.raises(urllib.error.HTTPError) as e:
        urllib.request.urlopen(url + "/nope", timeout=10)
    assert e.value.code == 404


def test_sigterm_stops_cleanly(server):
    p, _ = server
    p.send_signal(signal.SIGTERM)
    assert p.wait(10) == 0


@pytest.mark.gpu
def test_exporter_reports_mi355x(exe):
    r = subprocess.run([exe, "--once", "--hostname", "n0"], capture_output=True, text=True, timeout=60)
    rows = parse_exposition(r.stdout)
    names = {n for n, _, _ in rows}
    assert {"gpu_total_vram", "gpu_power_usage"} <= names, names
    total = [v for n, l, v in rows if n == "gpu_total_vram" and l["gpu_id"] == "0"][0]
    assert 280e9 / 2**20 < total <= 288 * 1024
    labels = [l for n, l, _ in rows if n == "gpu_power_usage" and l["gpu_id"] == "0"][0]
    # HIP's device name is empty on this ROCm; the probe names the board from sysfs / device id.
    assert labels["card_model"] == "AMD Instinct MI355X", labels
    assert re.fullmatch(r"[0-9A-F]{16}", labels["serial_number"]), labels
    slow = [v for n, l, v in rows if n == "gpu_junction_temperature_slowdown" and l["gpu_id"] == "0"]
    assert slow and 90 <= slow[0] <= 120, slow  # amd-smi: slowdown_hotspot_temperature 100 C
    part = [l for n, l, _ in rows if n == "gpu_partition_info"]
    assert part and part[0]["compute_partition"] in {"SPX", "DPX", "QPX", "CPX"}, part
    assert part[0]["memory_partition"] in {"NPS1", "NPS2", "NPS4", "NPS8"}, part
    one = subprocess.run([exe, "--once", "--hostname", "n0", "--device", "0", "--gpu-label", "7"],
                         capture_output=True, text=True, timeout=60)
    ids = {l["gpu_id"] for n, l, _ in parse_exposition(one.stdout)}
    assert ids == {"7"}
    time.sleep(0)


def test_exporter_process_and_device_relabel(exe):
    from headlamp_intel_gpu_plugin_amd.parallel.agent import (ExporterProcess, NodeAgent, Scraper, device_to_node,
                                                              live_series)

    p = ExporterProcess(hostname="host-a").start()
    try:
        assert "# TYPE gpu_power_usage gauge" in p.scrape()
    finally:
        p.stop()
    assert p.proc.returncode == 0
    # A host-wide exporter's device 0 belongs to rank 0's synthetic node.
    agent = NodeAgent("host-a", lambda: {"power_w": 321.0, "vram_total_b": 2.0 ** 30}).start()
    try:
        live = live_series(["mi355x-003"])
        s = Scraper([(agent.url, device_to_node({"0": "mi355x-003"}))], live, now=lambda: 100.0)
        s.scrape_once()
        assert s.scrapes == 1
        assert live[("mi355x-003", 0)]["gpu_power_usage"].at(100.0)[1] == 321.0
        assert live[("mi355x-003", 0)]["gpu_total_vram"].at(100.0)[1] == 1024.0
        assert device_to_node({"0": "n"})({"gpu_id": "5"}) is None
        # On the scrape grid (the ServiceMonitor's 15 s): a scrape just after a grid point is stamped with it; one
        # off the grid (the first, at start) keeps its time, so no value is dated seconds before it was read.
        clock = [120.02]
        aligned = Scraper([(agent.url, device_to_node({"0": "mi355x-003"}))], live, interval=15.0, now=lambda: clock[0],
                          align=True)
        aligned.scrape_once()
        assert live[("mi355x-003", 0)]["gpu_power_usage"].ts[-1] == 120.0
        clock[0] = 127.3
        aligned.scrape_once()
        assert live[("mi355x-003", 0)]["gpu_power_usage"].ts[-1] == 127.3
    finally:
        agent.stop()


# ---------------------------------------------------------------------------
# --sysfs-only: devices and xGMI links from the KFD topology, no HIP runtime
# ---------------------------------------------------------------------------

FIX = os.path.join(os.path.dirname(__file__), "fixtures", "mi355x")


def _kfd_nodes(path):
    """tests/fixtures/mi355x/kfd_topology.txt → [(node, props text, {link: props text})]."""
    nodes, cur, link = [], None, None
    for line in open(path):
        line = line.rstrip("\n")
        if line.startswith("== node "):
            cur = [int(line.split()[2]), [], {}]
            nodes.append(cur)
            link = None
        elif line.startswith("-- "):
            link = line[3:]
            cur[2][link] = []
        elif cur is not None and line and not line.startswith("#") and not line.startswith(("gpu_id ", "name ")):
            (cur[2][link] if link else cur[1]).append(line)
    return nodes


def _drm_cards():
    """tests/fixtures/mi355x/drm_cards.txt → [(card number, bdf)] in card order."""
    out = []
    for line in open(os.path.join(FIX, "drm_cards.txt")):
        if line.startswith("#") or not line.strip():
            continue
        f = line.split()
        out.append((int(f[0][4:]), f[3]))
    return sorted(out)


def _sysfs_tree(root, kfd_nodes):
    """DRM cards + PCI device dirs of the captured host, and the given KFD nodes."""
    for i, (card, bdf) in enumerate(_drm_cards()):
        d = root / "sys/bus/pci/devices" / bdf
        (d / "hwmon/hwmon0").mkdir(parents=True)
        (d / "vendor").write_text("0x1002\n")
        (d / "device").write_text("0x75a3\n")
        (d / "mem_info_vram_total").write_text(str(294896 * 1024 * 1024) + "\n")
        (d / "mem_info_vram_used").write_text(str((1000 + i) * 1024 * 1024) + "\n")
        (d / "gpu_busy_percent").write_text(f"{10 * i}\n")
        (d / "hwmon/hwmon0/power1_input").write_text(f"{(200 + i) * 1000000}\n")
        c = root / "sys/class/drm" / f"card{card}"
        c.mkdir(parents=True)
        os.symlink(d, c / "device")
    base = root / "sys/class/kfd/kfd/topology/nodes"
    for node, props, links in kfd_nodes:
        nd = base / str(node)
        nd.mkdir(parents=True)
        if props:  # an unreadable node (another container's GPU) has no properties for us
            (nd / "properties").write_text("\n".join(props) + "\n")
        for name, lp in links.items():
            (nd / name).mkdir(parents=True, exist_ok=True)
            if lp:
                (nd / name / "properties").write_text("\n".join(lp) + "\n")
    return root


def _scrape_sysfs_only(exe, root):
    env = dict(os.environ, AMDGPU_EXPORTER_SYSFS_ROOT=str(root))
    r = subprocess.run([exe, "--once", "--sysfs-only", "--hostname", "n0"], capture_output=True, text=True,
                       timeout=60, env=env)
    assert r.returncode == 0, r.stderr
    assert "sysfs-only" in r.stderr
    return parse_exposition(r.stdout)


def test_sysfs_only_enumerates_gpus_from_drm_cards(exe, tmp_path):
    # The KFD tree as captured in a 1-GPU container: only this container's GPU
    # node (2) is readable, so no link has two readable ends.
    rows = _scrape_sysfs_only(exe, _sysfs_tree(tmp_path, _kfd_nodes(os.path.join(FIX, "kfd_topology.txt"))))
    power = [(l["gpu_id"], l["pci_bus"], l["card_model"], v) for n, l, v in rows if n == "gpu_power_usage"]
    cards = _drm_cards()
    assert [p[0] for p in power] == [str(i) for i in range(8)]
    assert [p[1] for p in power] == [b for _, b in cards]  # card order: card0, card8, card16, ...
    assert all(p[2] == "AMD Instinct MI355X" for p in power)
    assert [p[3] for p in power] == [200.0 + i for i in range(8)]
    assert {v for n, l, v in rows if n == "gpu_total_vram"} == {294896.0}
    assert [v for n, l, v in rows if n == "gpu_gfx_activity"] == [10.0 * i for i in range(8)]
    assert not [1 for n, _, _ in rows if n == "gpu_xgmi_link_hops"]


def test_sysfs_only_reads_xgmi_links_from_a_readable_kfd_topology(exe, tmp_path):
    # Every GPU node readable (a pod whose device cgroup admits the render
    # nodes): node 2's captured properties as the template, each node at its
    # card's PCI address, every GPU linked to the 7 others (io_link type 11).
    # GPU 0 (KFD node 2) keeps its captured io_links verbatim: a PCIe link to
    # its CPU node, then xGMI to nodes 3..9 in that order. The others list a
    # PCIe link, then their peers ROTATED (GPU k: k+1, k+2, ... mod 8), so the
    # exporter's `neighbor` label must follow io_link order, not GPU index.
    # SYNTHETIC beyond node 2: the capture could read only its own GPU.
    captured = {n: (p, l) for n, p, l in _kfd_nodes(os.path.join(FIX, "kfd_topology.txt"))}
    template = [l for l in captured[2][0] if not l.startswith(("location_id ", "domain "))]
    xgmi_tmpl = next(lp for name, lp in captured[2][1].items() if lp and "type 11" in lp)
    pcie_tmpl = captured[2][1]["io_links/0"]
    nodes = [(0, captured[0][0], {}), (1, captured[1][0], {})]
    cards = _drm_cards()
    order = {}
    for k, (_, bdf) in enumerate(cards):
        bus, dev, fn = int(bdf[5:7], 16), int(bdf[8:10], 16), int(bdf[11], 16)
        props = template + [f"location_id {bus << 8 | dev << 3 | fn}", "domain 0"]
        if k == 0:
            links = {name: lp for name, lp in captured[2][1].items() if name.startswith("io_links")}
        else:
            links = {"io_links/0": pcie_tmpl}
            for j in ((k + d) % len(cards) for d in range(1, len(cards))):
                links[f"io_links/{len(links)}"] = [l if not l.startswith("node_to ") else f"node_to {j + 2}" for l in xgmi_tmpl]
        # expected neighbour order: the xGMI io_links' node_to, in io_link number order
        xg = [dict(x.split(" ", 1) for x in links[f"io_links/{i}"]) for i in range(len(links))]
        order[k] = [int(l["node_to"]) - 2 for l in xg if l["type"] == "11"]
        nodes.append((k + 2, props, links))
    assert order[0] == [1, 2, 3, 4, 5, 6, 7]  # the capture: node 2 → nodes 3..9
    assert order[3] == [4, 5, 6, 7, 0, 1, 2]
    rows = _scrape_sysfs_only(exe, _sysfs_tree(tmp_path, nodes))
    hops = {(l["gpu_id"], l["peer_gpu_id"]): v for n, l, v in rows if n == "gpu_xgmi_link_hops"}
    assert len(hops) == 56 and set(hops.values()) == {1.0}
    assert all((str(a), str(b)) in hops for a in range(8) for b in range(8) if a != b)
    neighbor = {(int(l["gpu_id"]), int(l["neighbor"])): int(l["peer_gpu_id"]) for n, l, v in rows if n == "gpu_xgmi_link_hops"}
    assert neighbor == {(a, k): order[a][k] for a in range(8) for k in range(7)}


def test_neighbor_numbers_count_links_to_unreadable_peers(exe, tmp_path):
    """A link whose peer this process cannot read is not exported, but it keeps its place: the next readable peer's
    `neighbor` is its io_link position among ALL xGMI links (what a per-neighbour series from another exporter counts)."""
    captured = {n: (p, l) for n, p, l in _kfd_nodes(os.path.join(FIX, "kfd_topology.txt"))}
    template = [l for l in captured[2][0] if not l.startswith(("location_id ", "domain "))]
    cards = _drm_cards()
    nodes = [(0, captured[0][0], {}), (1, captured[1][0], {})]
    readable = {0, 4}  # GPUs 0 and 4 only: GPU 0 reaches GPU 4 as its 4th xGMI neighbour (nodes 3,4,5 unreadable)
    for k, (_, bdf) in enumerate(cards):
        bus, dev, fn = int(bdf[5:7], 16), int(bdf[8:10], 16), int(bdf[11], 16)
        props = (template + [f"location_id {bus << 8 | dev << 3 | fn}", "domain 0"]) if k in readable else []
        links = {name: lp for name, lp in captured[2][1].items() if name.startswith("io_links")} if k == 0 else {}
        nodes.append((k + 2, props, links))
    rows = _scrape_sysfs_only(exe, _sysfs_tree(tmp_path, nodes))
    links = [(l["gpu_id"], l["peer_gpu_id"], l["neighbor"]) for n, l, v in rows if n == "gpu_xgmi_link_hops"]
    assert links == [("0", "4", "3")]


def test_captured_kfd_topology_links_this_gpu_to_seven_peers_over_xgmi():
    # What the capture itself shows about an MI355X: its GPU node has 7 xGMI
    # io_links (type 11, weight 15, 76 GB/s) and one PCIe link to its CPU node.
    nodes = {n: (p, l) for n, p, l in _kfd_nodes(os.path.join(FIX, "kfd_topology.txt"))}
    props = dict(l.split(" ", 1) for l in nodes[2][0])
    assert props["simd_count"] == "1024" and props["gfx_target_version"] == "90500"
    assert int(props["device_id"]) == 0x75A3 and props["lds_size_in_kb"] == "160" and props["num_xcc"] == "8"
    links = [dict(x.split(" ", 1) for x in lp) for name, lp in nodes[2][1].items() if name.startswith("io_links") and lp]
    xgmi = [l for l in links if l["type"] == "11"]
    assert len(xgmi) == 7 and {l["weight"] for l in xgmi} == {"15"} and {l["max_bandwidth"] for l in xgmi} == {"76000"}
    assert sorted(int(l["node_to"]) for l in xgmi) == list(range(3, 10))


def _start(exe, name):
    p = subprocess.Popen([exe, "--port", "0", "--bind", "127.0.0.1", "--hostname", name, "--sysfs-only"],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    line = p.stdout.readline()
    return p, int(line.split("127.0.0.1:")[1].split()[0])


def test_slow_client_does_not_block_scrapes(exe):
    """Peers trickling header bytes and peers that never read hold only their own sockets (one poll() loop, no
    worker threads): /healthz and /metrics answer at once next to them, and the trickling connections are dropped
    at the request deadline."""
    import socket

    p, port = _start(exe, "slow")
    try:
        slow = [socket.create_connection(("127.0.0.1", port)) for _ in range(64)]
        stalled = []
        for _ in range(8):
            s = socket.create_connection(("127.0.0.1", port))
            s.sendall(b"GET /metrics HTTP/1.1\r\nHost: x\r\n\r\n")  # never read
            stalled.append(s)
        t0 = time.time()
        for s in slow:
            s.sendall(b"G")
        for _ in range(3):
            for path in ("/healthz", "/metrics"):
                t = time.time()
                with urllib.request.urlopen(f"http://127.0.0.1:{port}{path}", timeout=5) as r:
                    body = r.read()
                assert time.time() - t < 0.5, path
                assert body == b"ok\n" if path == "/healthz" else b"# HELP" in body or body == b""
            for s in slow:
                try:
                    s.sendall(b"E")
                except OSError:
                    pass
            time.sleep(0.5)
        # The trickling connections are dropped at the deadline (~3 s), not held.
        slow[0].settimeout(10)
        try:
            data = slow[0].recv(100)
        except ConnectionResetError:
            data = b""
        assert data == b"" and time.time() - t0 < 8
        for s in slow + stalled:
            s.close()
    finally:
        p.send_signal(signal.SIGTERM)
        assert p.wait(15) == 0


def test_full_connection_table_drops_the_oldest_request_in_progress(exe):
    """At the connection limit (512) a new peer evicts the oldest connection still sending its request, so a
    scrape gets through however many idle sockets an attacker opens."""
    import resource
    import socket

    soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
    if min(soft, hard) < 1200:
        pytest.skip(f"needs ~600 client sockets (RLIMIT_NOFILE {soft})")
    p, port = _start(exe, "full")
    idle = []
    try:
        for _ in range(530):
            idle.append(socket.create_connection(("127.0.0.1", port)))
        time.sleep(0.2)
        t = time.time()
        with urllib.request.urlopen(f"http://127.0.0.1:{port}/healthz", timeout=5) as r:
            assert r.read() == b"ok\n"
        assert time.time() - t < 1.0
        # the oldest idle peers were the ones dropped
        idle[0].settimeout(2)
        try:
            assert idle[0].recv(10) == b""
        except ConnectionResetError:
            pass
    finally:
        for s in idle:
            s.close()
        p.send_signal(signal.SIGTERM)
        assert p.wait(15) == 0


def test_descriptor_limit_caps_the_connection_table(exe):
    """With a small RLIMIT_NOFILE the table is capped below it: idle peers past the cap evict older ones instead of
    making accept() fail with EMFILE (which would leave the listen socket readable and spin poll()), so scrapes
    still answer and the daemon stays idle on the CPU."""
    import resource
    import socket

    def small_limit():
        resource.setrlimit(resource.RLIMIT_NOFILE, (64, resource.getrlimit(resource.RLIMIT_NOFILE)[1]))

    p = subprocess.Popen([exe, "--port", "0", "--bind", "127.0.0.1", "--hostname", "fd", "--sysfs-only"],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, preexec_fn=small_limit)
    port = int(p.stdout.readline().split("127.0.0.1:")[1].split()[0])
    idle = []
    try:
        for _ in range(100):
            idle.append(socket.create_connection(("127.0.0.1", port)))
        time.sleep(0.3)

        def cpu_ticks():
            f = open(f"/proc/{p.pid}/stat").read().rsplit(")", 1)[1].split()
            return int(f[11]) + int(f[12])  # utime + stime

        before = cpu_ticks()
        time.sleep(1.0)
        assert cpu_ticks() - before < 30  # < 0.3 s of CPU in 1 s: no EMFILE spin
        for path in ("/healthz", "/metrics"):
            t = time.time()
            with urllib.request.urlopen(f"http://127.0.0.1:{port}{path}", timeout=5) as r:
                assert r.status == 200
            assert time.time() - t < 1.0, path
    finally:
        for s in idle:
            s.close()
        p.send_signal(signal.SIGTERM)
        assert p.wait(15) == 0


@pytest.mark.gpu
def test_sysfs_only_on_the_box_matches_the_hip_scrape(exe):
    """--sysfs-only (no HIP, what the unprivileged DaemonSet runs) sees every
    MI355X card of the host in sysfs; for the GPU HIP sees, the series agree."""
    hip = parse_exposition(subprocess.run([exe, "--once", "--hostname", "n0"], capture_output=True, text=True,
                                          timeout=60).stdout)
    r = subprocess.run([exe, "--once", "--sysfs-only", "--hostname", "n0"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    sysfs = parse_exposition(r.stdout)
    models = {l["pci_bus"]: l["card_model"] for n, l, _ in sysfs if n == "gpu_total_vram"}
    assert len(models) >= 1 and set(models.values()) == {"AMD Instinct MI355X"}, models
    hip_bus = [l["pci_bus"] for n, l, _ in hip if n == "gpu_total_vram"][0]
    assert hip_bus in models
    total = lambda rows, bus: [v for n, l, v in rows if n == "gpu_total_vram" and l["pci_bus"] == bus][0]
    assert total(sysfs, hip_bus) == total(hip, hip_bus)
    # Power / temperature of the visible GPU come from the same hwmon files.
    assert [v for n, l, v in sysfs if n == "gpu_junction_temperature" and l["pci_bus"] == hip_bus]
    print("sysfs-only GPUs:", len(models), "link series:", sum(1 for n, _, _ in sysfs if n == "gpu_xgmi_link_hops"))


def test_garbage_requests_do_not_break_the_daemon(exe):
    """Random bytes, truncated request lines, huge headers, pipelined junk: each gets a 4xx or a close, and the
    daemon keeps serving."""
    import random
    import socket

    p, port = _start(exe, "fuzz")
    rnd = random.Random(7)
    payloads = [b"", b"\r\n\r\n", b"GET\r\n\r\n", b"GET / HTTP/1.1", b"POST /metrics HTTP/1.1\r\n\r\n",
                b"GET /" + b"a" * 20000 + b" HTTP/1.1\r\n\r\n", b"\x00\xff" * 100 + b"\r\n\r\n",
                b"GET /healthz HTTP/1.1\r\n\r\nGET /metrics HTTP/1.1\r\n\r\n"]
    payloads += [bytes(rnd.getrandbits(8) for _ in range(rnd.randint(1, 3000))) for _ in range(40)]
    try:
        for data in payloads:
            with socket.create_connection(("127.0.0.1", port), timeout=5) as s:
                try:
                    s.sendall(data)
                    s.shutdown(socket.SHUT_WR)
                    s.recv(65536)
                except OSError:
                    pass
        with urllib.request.urlopen(f"http://127.0.0.1:{port}/healthz", timeout=5) as r:
            assert r.read() == b"ok\n"
        assert p.poll() is None
    finally:
        p.send_signal(signal.SIGTERM)
        assert p.wait(15) == 0


def test_half_closed_client_still_gets_its_answer(exe):
    """A peer that sends a whole request and then shuts its write side (`nc -N`, HTTP/1.0 probes) is answered; one
    that half-closes mid-request is dropped without an answer."""
    import socket

    p, port = _start(exe, "halfclose")
    try:
        for path, expect in ((b"/healthz", b"ok\n"), (b"/metrics", b"")):
            with socket.create_connection(("127.0.0.1", port), timeout=5) as s:
                s.sendall(b"GET " + path + b" HTTP/1.0\r\n\r\n")
                s.shutdown(socket.SHUT_WR)
                data = b""
                while True:
                    chunk = s.recv(65536)
                    if not chunk:
                        break
                    data += chunk
            assert data.startswith(b"HTTP/1.1 200"), data[:80]
            assert data.endswith(expect)
        with socket.create_connection(("127.0.0.1", port), timeout=5) as s:
            s.sendall(b"GET /healthz HTTP/1.0\r\n")  # no blank line: incomplete
            s.shutdown(socket.SHUT_WR)
            assert s.recv(100) == b""
        assert p.poll() is None
    finally:
        p.send_signal(signal.SIGTERM)
        assert p.wait(15) == 0


@pytest.fixture(scope="module")
def asan(tmp_path_factory):
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import asan_exporter

    return asan_exporter, asan_exporter.build(str(tmp_path_factory.mktemp("asan")))


def test_http_serving_is_clean_under_asan_and_ubsan(asan):
    """Host-code AddressSanitizer + UBSan build of the daemon (tools/asan_exporter.py): fuzzed requests, slow
    peers, scrapes and shutdown produce no report and no leak."""
    mod, exe = asan
    ok, rc, err = mod.drive(exe)
    assert ok, (rc, err[-3000:])


def test_sysfs_and_kfd_parsing_is_clean_under_asan_and_ubsan(asan, tmp_path):
    """The probe's sysfs / KFD readers (probe_core.h) under the sanitizers, on the captured host's trees: the
    1-GPU-container KFD view and a fully readable 8-GPU one."""
    _, exe = asan
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    captured = _kfd_nodes(os.path.join(FIX, "kfd_topology.txt"))
    for name, nodes in (("one", captured), ("none", [])):
        root = _sysfs_tree(tmp_path / name, nodes)
        r = subprocess.run([exe, "--once", "--sysfs-only", "--hostname", "n0"], capture_output=True, text=True,
                           timeout=120, env=dict(env, AMDGPU_EXPORTER_SYSFS_ROOT=str(root)))
        assert r.returncode == 0 and "runtime error" not in r.stderr and "Sanitizer" not in r.stderr, r.stderr[-3000:]
        assert "gpu_power_usage" in r.stdout
