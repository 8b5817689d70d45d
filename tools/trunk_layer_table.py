"""Per-launch table of the inference trunk from tools/gpu_r05x.sh (rocprofv3 --pmc passes p1..p5 + a kernel trace of
`bench.py --steps 2 --warmup 1 --stream-groups 1`): for every conv launch of the LAST bench step (stem .. proj) --
duration (kernel trace), MFMA busy per SIMD, wait / issue-stall shares of the wave cycles, VALU and LDS instructions per
MFMA, L2 hit rate and HBM bytes (FETCH x2 + WRITE, the gfx950 correction of MI355X_MICROARCH.md) and their rate.

    python tools/trunk_layer_table.py gpurun_out/<tag> > profiles/<tag>_trunk_layer_table.txt

Dispatch ids pair the passes (each pass runs the same launch sequence).  Counters are summed over a dispatch's rows;
SQ cycle counters count per 4 cycles except SQ_VALU_MFMA_BUSY_CYCLES; GRBM_GUI_ACTIVE is summed over the 8 XCDs.
"""
import collections
import csv
import glob
import os
import sys

QUAD = {"SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
        "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VALU"}
N_SIMD = 256 * 4


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0][:44]


def main():
    root = sys.argv[1]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    npass = collections.defaultdict(lambda: collections.defaultdict(int))
    names = {}
    for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
        one = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            d = int(r["Dispatch_Id"])
            one[d][r["Counter_Name"]] += float(r["Counter_Value"])
            names[d] = r["Kernel_Name"]
        for d, c in one.items():  # counters repeated in several passes (SQ_WAVES, GRBM_GUI_ACTIVE): averaged
            for k, v in c.items():
                per[d][k] += v
                npass[d][k] += 1
    for d, c in per.items():
        for k in c:
            c[k] /= npass[d][k]
    trace = {}
    for f in glob.glob(os.path.join(root, "kt", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            trace[int(r["Dispatch_Id"])] = (r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3,
                                            r.get("Grid_Size_X", r.get("Grid_Size", "")))
    ids = sorted(trace)
    stems = [d for d in ids if "stem" in trace[d][0]]
    warps = [d for d in ids if "warp_fuse" in trace[d][0]]
    if not stems or not warps:
        sys.exit("no stem / warp launches in the trace")
    first, last = stems[-1], warps[-1]
    print(f"{'kernel':44s} {'grid':>9s} {'us':>8s} {'mfma':>5s} {'wait':>5s} {'stall':>5s} {'valu/mf':>7s} "
          f"{'lds/mf':>6s} {'L2hit':>5s} {'HBM MB':>8s} {'TB/s':>5s}")
    tot_us = tot_mb = 0.0
    for d in ids:
        if d < first or d >= last:
            continue
        nm, us, grid = trace[d]
        if "conv" not in nm and "stem" not in nm and "maxpool" not in nm:
            continue
        c = per.get(d, {})
        w = c.get("SQ_WAVES", 0.0) or 1.0
        cyc = c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0 or 1.0
        mf = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        wc = c.get("SQ_WAVE_CYCLES", 0.0) * 4 or 1.0
        n_mfma = mf / 32.0 or 1.0  # 32-cycle MFMAs (v_mfma_f32_32x32x16_*); the exact-f32 stem's are 64
        fetch = 2.0 * c.get("FETCH_SIZE", 0.0) * 1024
        write = c.get("WRITE_SIZE", 0.0) * 1024
        hit, miss = c.get("TCC_HIT_sum", 0.0), c.get("TCC_MISS_sum", 0.0)
        mb = (fetch + write) / 1e6
        tot_us += us
        tot_mb += mb
        print(f"{short(nm):44s} {grid:>9s} {us:8.1f} {mf / (N_SIMD * cyc):5.2f} {c.get('SQ_WAIT_ANY', 0) * 4 / wc:5.2f} "
              f"{c.get('SQ_WAIT_INST_ANY', 0) * 4 / wc:5.2f} {c.get('SQ_INSTS_VALU', 0) / n_mfma:7.2f} "
              f"{c.get('SQ_INSTS_LDS', 0) / n_mfma:6.2f} {hit / max(hit + miss, 1):5.2f} {mb:8.1f} "
              f"{mb / 1e6 / (us * 1e-6) if us else 0:5.2f}")
    print(f"{'total (conv + max-pool launches of one step)':44s} {'':>9s} {tot_us:8.1f} {'':>5s} {'':>5s} {'':>5s} "
          f"{'':>7s} {'':>6s} {'':>5s} {tot_mb:8.1f}")


if __name__ == "__main__":
    main()
