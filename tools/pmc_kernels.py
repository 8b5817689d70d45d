"""Per-kernel counter summary of a rocprofv3 --pmc run directory tree (p1, p2, ... from tools/gpu_r05q.sh):
    python tools/pmc_kernels.py gpurun_out/<tag> [name-substring]
Per dispatch of each kernel: counters summed over the dispatch's rows, then per-wave values (cycles x4 for the
SQ cycle counters, which count per 4 cycles on gfx9), averaged over the kernel's dispatches."""
import collections
import csv
import glob
import os
import sys

QUAD = {"SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
        "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VALU", "SQ_VALU_MFMA_BUSY_CYCLES"}


def main():
    root, sub = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        names = {}
        for r in csv.DictReader(open(f)):
            if sub and sub not in r["Kernel_Name"]:
                continue
            d = int(r["Dispatch_Id"])
            per[d][r["Counter_Name"]] += float(r["Counter_Value"])
            names[d] = (r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:50] + " grid "
                        + r.get("Grid_Size", "?"))
        for d, c in per.items():
            w = c.get("SQ_WAVES", 0) or 1
            for k, v in c.items():
                agg[names[d]][k].append(v if k in ("GRBM_GUI_ACTIVE", "SQ_WAVES", "FETCH_SIZE", "WRITE_SIZE") or k.startswith("TCC") else
                                        v * (4 if k in QUAD else 1) / w)
    for n, c in agg.items():
        if "conv" not in n and "wgrad" not in n and sub == "":
            continue
        print(n)
        for k in sorted(c):
            v = c[k]
            print(f"    {k:28s} {sum(v) / len(v):14.1f}   (n={len(v)})")


if __name__ == "__main__":
    main()
