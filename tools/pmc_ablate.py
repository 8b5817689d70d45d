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
        g = lambda k, s=1.0: f"{s * c[k] / w:8.0f}" if k in c else "       -"
        print(f"{os.path.basename(d):>5}: gui {gui:9.0f} cyc  wave-cyc {g('SQ_WAVE_CYCLES', 4)}  valu {g('SQ_INSTS_VALU')}  "
              f"valu-cyc {g('SQ_ACTIVE_INST_VALU', 4)}  lds {g('SQ_INSTS_LDS')}  lds-cyc {g('SQ_ACTIVE_INST_LDS', 4)}  "
              f"conflicts {g('SQ_LDS_BANK_CONFLICT')}  salu {g('SQ_INSTS_SALU')}  smem {g('SQ_INSTS_SMEM')}  "
              f"wait-any {g('SQ_WAIT_ANY', 4)}  wait-inst {g('SQ_WAIT_INST_ANY', 4)}  (per wave)")


if __name__ == "__main__":
    main()
