"""Summarise tools/gpu_pmc_cmd.sh output for the kernels whose name contains a substring: counters of the last
dispatch, clock, waits and instruction mix per wave.  python tools/pmc_kernel.py gpurun_out/<tag> <substring>"""
import collections
import csv
import glob
import sys


def load(d, sub):
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f[0])):
        if sub in r["Kernel_Name"]:
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    return per[max(per)] if per else {}


def main():
    root, sub = sys.argv[1], sys.argv[2]
    c = dict(load(root + "/p1", sub))
    c.update(load(root + "/p2", sub))
    us = None
    for r in csv.DictReader(open(glob.glob(root + "/kt/**/*kernel_stats.csv", recursive=True)[0])):
        if sub in r["Name"]:
            us = float(r["AverageNs"]) / 1e3
            print(f"{r['Name'][:90]}: {r['Calls']} calls, avg {us:.1f} us")
    if not c or us is None:
        return
    waves = c["SQ_WAVES"]
    gui = c["GRBM_GUI_ACTIVE"] / 8.0
    wc = c["SQ_WAVE_CYCLES"]
    print(f"clock {gui / us / 1e3:.2f} GHz  waves {waves:.0f}  cycles/wave {4 * wc / waves:.0f}")
    print(f"active {c['SQ_ACTIVE_INST_ANY'] / wc:.3f}  issue-stall {c['SQ_WAIT_INST_ANY'] / wc:.3f} "
          f"(lds {c['SQ_WAIT_INST_LDS'] / wc:.3f})  wait {c['SQ_WAIT_ANY'] / wc:.3f}")
    print(f"per wave: valu {c['SQ_INSTS_VALU'] / waves:.0f}  salu {c['SQ_INSTS_SALU'] / waves:.0f}  "
          f"lds {c['SQ_INSTS_LDS'] / waves:.0f}  vmem {c['SQ_INSTS_VMEM'] / waves:.0f}")
    simd_cycles = gui * 256 * 4
    print(f"VALU busy {4 * c['SQ_ACTIVE_INST_VALU'] / simd_cycles:.3f} of SIMD cycles; LDS bank-conflict cycles per CU "
          f"{c['SQ_LDS_BANK_CONFLICT'] / 256:.0f} of {gui:.0f}")


if __name__ == "__main__":
    main()
