"""tools/ab_cold_open.py: how a CPU profile's self time is attributed to the A/B table's rows
(profiles/r6_ab_cold1k_cpu.md). The run itself needs two worktrees and minutes of CPU; these pin the accounting."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import ab_cold_open as ab  # noqa: E402


def test_every_plugin_module_has_one_row():
    base = "file:///tmp/ab-ee2699e/"
    assert ab.group_of(base + "src/api/amdPods.js", "isGpuRequestingPod") == "arrival facts"
    assert ab.group_of(base + "src/api/operatorFacts.js", "operatorPodFacts") == "arrival facts"
    assert ab.group_of(base + "src/api/clusterIndex.js", "buildClusterIndex") == "cluster index"
    assert ab.group_of(base + "src/api/listCache.js", "firstLoad") == "lists + store"
    assert ab.group_of(base + "src/api/telemetry.js", "joinExporterResults") == "telemetry client"
    assert ab.group_of(base + "src/view/pages/nodes.js", "nodesView") == "views"
    assert ab.group_of(base + "src/view/ir.js", "section") == "views"
    assert ab.group_of(base + "src/plugin.js", "anything") == "other plugin"
    assert ab.group_of(base + "bench/common.js", "decode") == "bench: response decode"
    assert ab.group_of(base + "bench/driver.js", "main") == "bench: other"
    assert ab.group_of("node:internal/streams/readable", "read") == "Node internals / V8"
    assert ab.group_of("", "(garbage collector)") == "GC"
    assert ab.group_of("", "(idle)") == "idle / program"
    # the plugin total sums exactly the plugin rows
    plugin_rows = {n for n, _ in ab.GROUPS[:5]}
    assert plugin_rows == {"arrival facts", "cluster index", "lists + store", "telemetry client", "views"}


def test_self_time_is_the_sum_of_each_sample_delta(tmp_path):
    """A .cpuprofile's samples[i] ran for timeDeltas[i] µs: the time goes to that node's own frame, not its callers."""
    prof = {
        "nodes": [
            {"id": 1, "callFrame": {"functionName": "(root)", "url": "", "lineNumber": 0}},
            {"id": 2, "callFrame": {"functionName": "buildClusterIndex", "url": "file:///r/src/api/clusterIndex.js", "lineNumber": 265}},
            {"id": 3, "callFrame": {"functionName": "podFacts", "url": "file:///r/src/api/clusterIndex.js", "lineNumber": 185}},
            {"id": 4, "callFrame": {"functionName": "decode", "url": "file:///r/bench/common.js", "lineNumber": 9}},
            {"id": 5, "callFrame": {"functionName": "(garbage collector)", "url": "", "lineNumber": 0}},
        ],
        "samples": [2, 3, 3, 4, 5, 2],
        "timeDeltas": [1000, 500, 1500, 4000, 250, 1000],
    }
    f = tmp_path / "x.cpuprofile"
    f.write_text(json.dumps(prof))
    got = ab.self_times(str(f))
    assert got == {"cluster index": 4.0, "bench: response decode": 4.0, "GC": 0.25}
    top = ab.top_functions(str(f), 2)
    assert top == [("buildClusterIndex (api/clusterIndex.js:266)", 2.0), ("podFacts (api/clusterIndex.js:186)", 2.0)]
