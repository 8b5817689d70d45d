"""Summarise tools/gpu_conv_pmc.sh output: per layer, the SQ counters of its last conv launch.

python tools/pmc_summary.py gpurun_out/<tag>
MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x CUs x 4 SIMDs) (busy cycles are per SIMD, GUI per XCD
summed over 8 XCDs -> divide by 8 for wall cycles); clock = GRBM_GUI_ACTIVE / 8 / kernel time.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def last_launch(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        return None, None
    per = defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(f[0])):
        if "k_conv" not in r["Kernel_Name"] and "k_stem" not in r["Kernel_Name"]:
            continue
        did = int(r["Dispatch_Id"])
        per[did][r["Counter_Name"]] = per[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[did] = r["Kernel_Name"][:60]
    if not per:
        return None, None
    did = max(per)
    return per[did], names[did]


def main():
    root = sys.argv[1]
    for p1 in sorted(glob.glob(os.path.join(root, "p1_*"))):
        if not os.path.isdir(p1):
            continue
        L = os.path.basename(p1)[3:]
        c1, name = last_launch(p1)
        c2, _ = last_launch(os.path.join(root, "p2_" + L))
        t = open(os.path.join(root, f"time_{L}.txt")).read().strip().splitlines()[-1]
        us = float(t.split()[1])
        if c1 is None:
            print(L, "no counters")
            continue
        gui = c1["GRBM_GUI_ACTIVE"] / 8.0
        clk = gui / (us * 1e-6) / 1e9
        simd = 256 * 4
        mfma = c1["SQ_VALU_MFMA_BUSY_CYCLES"] / (gui * simd)
        wc = c1["SQ_WAVE_CYCLES"]
        print(f"{L:9s} {t.split(None, 1)[1]}")
        print(f"   clock {clk:.2f} GHz  MFMA busy {mfma:.3f}  waves {c1['SQ_WAVES']:.0f}  "
              f"wait_any {c1['SQ_WAIT_ANY'] / wc:.3f} wait_inst {c1['SQ_WAIT_INST_ANY'] / wc:.3f} "
              f"(lds {c1['SQ_WAIT_INST_LDS'] / wc:.3f}) active {c1['SQ_ACTIVE_INST_ANY'] / wc:.3f}  [{name}]")
        if c2:
            print(f"   valu {c2['SQ_INSTS_VALU']:.3g} lds {c2['SQ_INSTS_LDS']:.3g} salu {c2['SQ_INSTS_SALU']:.3g} "
                  f"bank_conflict {c2['SQ_LDS_BANK_CONFLICT']:.3g} active_lds {c2['SQ_ACTIVE_INST_LDS']:.3g}")


if __name__ == "__main__":
    main()
