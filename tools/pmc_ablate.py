"""Per-variant fused-warp counters from tools/gpu_r05c.sh: python tools/pmc_ablate.py gpurun_out/<tag>"""
import collections
import csv
import glob
import os
import sys


def main():
    root = sys.argv[1]
    for d in sorted(glob.glob(os.path.join(root, "v*")), key=lambda p: int(os.path.basename(p)[1:]) if
                    os.path.basename(p)[1:].isdigit() else 999):
        if not os.path.isdir(d):
            continue
        f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
        if not f:
            continue
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f[0])):
            if "warp_fuse" in r["Kernel_Name"]:
                per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        if not per:
            continue
        c = per[max(per)]
        w = c["SQ_WAVES"]
        gui = c["GRBM_GUI_ACTIVE"] / 8.0
        print(f"{os.path.basename(d):>5}: gui {gui:9.0f} cyc  valu/wave {c['SQ_INSTS_VALU'] / w:7.0f}  "
              f"valu-cyc/wave {4 * c['SQ_ACTIVE_INST_VALU'] / w:8.0f}  lds/wave {c['SQ_INSTS_LDS'] / w:6.0f}  "
              f"lds-cyc/wave {4 * c['SQ_ACTIVE_INST_LDS'] / w:7.0f}  conflicts/wave {c['SQ_LDS_BANK_CONFLICT'] / w:6.0f}  "
              f"wave-cyc {4 * c['SQ_WAVE_CYCLES'] / w:8.0f}")


if __name__ == "__main__":
    main()
