"""Summarise a rocprofv3 --kernel-trace --stats run into profiles/<name>.md.

    python tools/prof_summary.py gpurun_out/prof profiles/r1_bench_c2.md [steps]

Reads the *kernel_stats.csv (per-kernel totals) and *kernel_trace.csv
(per-dispatch) files, or rocprofv3's default *results.db (rocpd SQLite), groups kernels by short name, and reports time per step
and the average duration of the GIN scatter-add kernel (k_gine_agg_fwd), which
bench.py's HIP-event roofline must agree with.
"""
from __future__ import annotations

import csv
import re
import sys
from collections import defaultdict
from pathlib import Path


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\(.*", "", name)
    return name[:110]


def main():
    src = Path(sys.argv[1])
    dst = Path(sys.argv[2])
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else None
    stats = sorted(src.rglob("*kernel_stats.csv"))
    trace = sorted(src.rglob("*kernel_trace.csv"))
    rows = []
    agg_durs = []
    dbs = sorted(src.rglob("*results.db"))
    if not stats and dbs:
        # rocprofv3's default rocpd (SQLite) output: one row per dispatch
        import sqlite3
        con = sqlite3.connect(str(dbs[0]))
        per = defaultdict(list)
        for name, t0, t1 in con.execute(
                "select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d "
                "join rocpd_info_kernel_symbol s on d.kernel_id = s.id"):
            per[name].append(t1 - t0)
        tot_all = sum(sum(v) for v in per.values()) or 1
        for name, ds in per.items():
            rows.append((short(name), len(ds), float(sum(ds)), sum(ds) / len(ds),
                         100.0 * sum(ds) / tot_all))
            if "k_gine_agg_fwd" in name:
                agg_durs += ds
    if stats:
        with open(stats[0]) as f:
            for r in csv.DictReader(f):
                rows.append((short(r["Name"]), int(r["Calls"]), float(r["TotalDurationNs"]),
                             float(r["AverageNs"]), float(r["Percentage"])))
    agg = defaultdict(lambda: [0, 0.0])
    for n, c, tot, avg, pct in rows:
        agg[n][0] += c
        agg[n][1] += tot
    total = sum(v[1] for v in agg.values())
    lines = [f"# rocprofv3 kernel summary — {src}", ""]
    if agg_durs:
        lines.append(f"k_gine_agg_fwd: {len(agg_durs)} dispatches, average "
                     f"{sum(agg_durs)/len(agg_durs)/1e3:.2f} us, min {min(agg_durs)/1e3:.2f} us, "
                     f"max {max(agg_durs)/1e3:.2f} us")
        lines.append("")
    if trace:
        durs = []
        with open(trace[0]) as f:
            for r in csv.DictReader(f):
                if "k_gine_agg_fwd" in r["Kernel_Name"]:
                    durs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        if durs:
            lines.append(f"k_gine_agg_fwd: {len(durs)} dispatches, average {sum(durs)/len(durs)/1e3:.2f} us, "
                         f"min {min(durs)/1e3:.2f} us, max {max(durs)/1e3:.2f} us")
            lines.append("")
    lines.append(f"total kernel time {total/1e6:.2f} ms" +
                 (f" over the whole run; {steps} timed + warm-up steps" if steps else ""))
    lines.append("")
    lines.append("| kernel | calls | total ms | avg us | % |")
    lines.append("|---|---|---|---|---|")
    for n, (c, tot) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        lines.append(f"| `{n}` | {c} | {tot/1e6:.3f} | {tot/c/1e3:.2f} | {100*tot/total:.1f} |")
    dst.parent.mkdir(parents=True, exist_ok=True)
    dst.write_text("\n".join(lines) + "\n")
    print("\n".join(lines[:40]))


if __name__ == "__main__":
    main()
