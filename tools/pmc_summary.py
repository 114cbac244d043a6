#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc databases: mean counter value per dispatch, per kernel.

    python tools/pmc_summary.py gpurun_out/pmc/sq/sq_results.db [more.db ...] [--md]

Also derives, when the counters are present: MFMA utilisation
(SQ_VALU_MFMA_BUSY_CYCLES summed over the chip ÷ SIMD-cycles available, where
SQ_BUSY_CYCLES is summed over the 32 shader engines of an MI355X, each with
32 SIMDs), the effective shader clock (busy cycles per SE ÷ kernel time),
LDS bank-conflict share (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE), L2 hit rate
and HBM bytes (TCC_EA0_RDREQ x 128 B — gfx950 tallies a 128-B request as one
64-B unit, MI355X_MICROARCH.md §HBM — and TCC_EA0_WRREQ x 64 B).
"""
import argparse
import re
import sqlite3
from collections import defaultdict


N_SE = 32  # shader engines on an MI355X (8 XCDs); one counter instance each
SIMDS_PER_SE = 256 * 4 // N_SE


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    n = re.sub(r"\(.*", "", n)
    return n[:60]


def collect(paths):
    vals = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [value per dispatch]
    dur = defaultdict(dict)
    for p in paths:
        db = sqlite3.connect(p)
        for kname, dispatch, counter, value, d in db.execute(
                "select kernel_name, dispatch_id, counter_name, sum(value), max(duration) from counters_collection "
                "group by dispatch_id, counter_name"):
            k = short(kname)
            vals[k][counter].append(value)
            dur[k][dispatch] = d
    return vals, dur


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dbs", nargs="+")
    ap.add_argument("--md", action="store_true")
    a = ap.parse_args()
    vals, dur = collect(a.dbs)
    counters = sorted({c for k in vals for c in vals[k]})
    rows = []
    for k in sorted(vals, key=lambda k: -sum(dur[k].values())):
        if not any(s in k for s in ("gemm", "triad", "Cijk")):
            continue
        m = {c: sum(v) / len(v) for c, v in vals[k].items()}
        derived = {}
        mean_ns = sum(dur[k].values()) / max(1, len(dur[k]))
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and m.get("SQ_BUSY_CYCLES"):
            derived["mfma_util"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["SQ_BUSY_CYCLES"] * SIMDS_PER_SE)
        if m.get("SQ_BUSY_CYCLES") and mean_ns > 0:
            derived["clock_GHz"] = m["SQ_BUSY_CYCLES"] / N_SE / mean_ns
        if "SQ_LDS_BANK_CONFLICT" in m and m.get("SQ_LDS_IDX_ACTIVE"):
            derived["lds_conflict"] = m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"]
        if m.get("TCC_HIT_sum") is not None and m.get("TCC_MISS_sum") is not None:
            derived["l2_hit"] = m["TCC_HIT_sum"] / max(1.0, m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
        if "TCC_EA0_RDREQ_sum" in m:
            derived["hbm_read_GB"] = m["TCC_EA0_RDREQ_sum"] * 128 / 1e9
        if "TCC_EA0_WRREQ_sum" in m:
            derived["hbm_write_GB"] = m["TCC_EA0_WRREQ_sum"] * 64 / 1e9
        rows.append((k, len(dur[k]), m, derived))
    if a.md:
        dcols = ["mfma_util", "clock_GHz", "lds_conflict", "l2_hit", "hbm_read_GB", "hbm_write_GB"]
        print("| kernel | dispatches | " + " | ".join(dcols) + " | " + " | ".join(counters) + " |")
        print("|---|---:|" + "---:|" * (len(dcols) + len(counters)))
        for k, n, m, d in rows:
            dv = [f"{d[c]:.3f}" if c in d else "—" for c in dcols]
            cv = [f"{m[c]:.4g}" if c in m else "—" for c in counters]
            print(f"| `{k}` | {n} | " + " | ".join(dv) + " | " + " | ".join(cv) + " |")
    else:
        for k, n, m, d in rows:
            print(k, n, {c: round(v, 3) for c, v in d.items()})


if __name__ == "__main__":
    main()
