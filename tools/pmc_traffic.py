"""Per-launch HBM traffic of the bench's dominant kernels from rocprofv3 --pmc passes.

Usage: python tools/pmc_traffic.py <fetch_dir> <write_dir> <out.json> [stem_launches_per_step | k4] [arith]

k4 (bench.py --backbone efficientnet_b3): "conv" is every native encoder launch of a step (stem, pointwise, depthwise,
SE gate, proj: what the K4 line's HBM roofline times), steps counted by the fused-warp launches (one per step).

Inputs are the run_counter_collection.csv files of two separate passes
(`--pmc FETCH_SIZE` and `--pmc WRITE_SIZE`) over the same `bench.py` command.
Corrections (MI355X_MICROARCH.md, HBM section): counters are in KiB; on gfx950
FETCH_SIZE reports half the bytes of wide (16 B/lane) coalesced reads, so it
is doubled.  WRITE_SIZE is exact for 16-B/lane stores; the warp's 4-B/lane
stores are uncalibrated (noted in the output).
The conv figure is per bench step (all backbone conv launches of one frame,
steps counted by the stem launches: one per image group, ResNet.stream_groups = 2 by
default); the warp figure is per launch.  The chained bottleneck kernels store 4 B/lane
(their WRITE_SIZE share is uncalibrated, like the warp's).
"""
import csv
import json
import sys
from collections import defaultdict


def family(name: str, k4: bool = False) -> str:
    if "warp_fuse" in name:
        return "warp"
    if "k_conv" in name or "k_stem" in name:
        return "conv"
    if k4 and any(k in name for k in ("k_pw_", "k_dwconv", "k_se_gate", "k_chan_scale")):
        return "conv"
    return "other"


def main():
    fdir, wdir, out = sys.argv[1:4]
    k4 = len(sys.argv) > 4 and sys.argv[4] == "k4"
    groups = 1 if k4 else int(sys.argv[4]) if len(sys.argv) > 4 else 2
    arith = sys.argv[5] if len(sys.argv) > 5 else "bf16x6"  # bench.py --conv-arith of the profiled command
    tot = defaultdict(float)
    n = defaultdict(int)
    steps = 0
    for cnt, d in (("FETCH_SIZE", fdir), ("WRITE_SIZE", wdir)):
        for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
            if r["Counter_Name"] != cnt:
                continue
            fam = family(r["Kernel_Name"], k4)
            tot[(fam, cnt)] += float(r["Counter_Value"]) * 1024.0
            if cnt == "FETCH_SIZE":
                n[fam] += 1
                if k4:
                    steps += "warp_fuse" in r["Kernel_Name"]  # one fused warp per step
                else:
                    steps += "k_stem" in r["Kernel_Name"] and "seams" not in r["Kernel_Name"]  # one stem per group
    res = {}
    steps //= groups
    for fam, per in (("conv", steps), ("warp", n["warp"])):
        if per == 0:
            continue
        fetch = 2.0 * tot[(fam, "FETCH_SIZE")] / per
        write = tot[(fam, "WRITE_SIZE")] / per
        res[fam] = {"fetch_bytes": round(fetch), "write_bytes": round(write), "traffic_bytes": round(fetch + write),
                    "per": "bench step" if fam == "conv" else "launch", "samples": per}
    res["note"] = ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes; FETCH x2 (gfx950 wide-read "
                   "correction), KiB -> bytes; warp and chained-conv stores are 4 B/lane (WRITE_SIZE uncalibrated for "
                   "that width)")
    res["conv_arith"] = arith
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
