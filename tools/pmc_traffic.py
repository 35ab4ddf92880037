"""HBM traffic per launch of the GIN scatter-add from rocprofv3 PMC passes.

    python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write profiles/r1_pmc_gine_agg.json

Inputs are two separate rocprofv3 runs (TCC slots do not fit both counters in
one pass): ``--pmc FETCH_SIZE`` and ``--pmc WRITE_SIZE``, both restricted to
k_gine_agg_fwd.  Per MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reports exactly half the bytes of a wide coalesced
streaming read (16 B per lane — this kernel's float4 gathers), so it is
doubled; WRITE_SIZE is exact for 16-B-per-lane stores.  Infinity-Cache hits are
counted, so this is memory-side (fabric) traffic, an upper bound on HBM bytes.
"""
from __future__ import annotations

import csv
import json
import statistics
import sys
from pathlib import Path

KERNEL = "k_gine_agg_fwd"


def read_counter(d: Path, name: str):
    vals = []
    for f in sorted(d.rglob("*counter_collection.csv")):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if KERNEL in r.get("Kernel_Name", "") and r.get("Counter_Name") == name:
                    vals.append(float(r["Counter_Value"]))
    return vals


def main():
    fetch_dir, write_dir, out = Path(sys.argv[1]), Path(sys.argv[2]), Path(sys.argv[3])
    fetch = read_counter(fetch_dir, "FETCH_SIZE")
    write = read_counter(write_dir, "WRITE_SIZE")
    if not fetch or not write:
        sys.exit(f"no {KERNEL} counter rows found (fetch {len(fetch)}, write {len(write)})")
    f_kib = statistics.median(fetch)
    w_kib = statistics.median(write)
    res = {
        "kernel": KERNEL,
        "dispatches": {"fetch_pass": len(fetch), "write_pass": len(write)},
        "FETCH_SIZE_KiB_median": f_kib,
        "WRITE_SIZE_KiB_median": w_kib,
        "correction": "FETCH_SIZE x2 (gfx950, 16-B coalesced reads); WRITE_SIZE x1",
        "hbm_bytes_per_launch": int((2 * f_kib + w_kib) * 1024),
    }
    out.write_text(json.dumps(res, indent=1))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
