"""Per-kernel counter table from rocprofv3 --pmc pass directories (any number of passes of the same command).

    python tools/pmc_table.py gpurun_out/<tag>/<pass dir> [<pass dir> ...] [--filter REGEX]

Counters are summed over all dispatches of a (kernel, grid) pair within each pass, then combined across passes
(GRBM_GUI_ACTIVE / SQ_WAVES averaged where several passes hold them).  Derived columns (MI355X_MICROARCH.md §PMC):
  mfma   SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)      (MFMA busy per SIMD)
  wait   SQ_WAIT_ANY / SQ_WAVE_CYCLES, stall SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES, lds_st SQ_WAIT_INST_LDS / ...
  valu/mf, lds/mf   SQ_INSTS_VALU or SQ_INSTS_LDS per MFMA (MFMA count = MFMA busy cycles / 32)
  vmem/mf, salu/mf  likewise; bank  SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS
"""
import collections
import csv
import glob
import os
import re
import sys


def load(d):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            key = (name[:52], r.get("Grid_Size", r.get("Grid_Size_X", "")))
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
    return per


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    filt = None
    if "--filter" in sys.argv:
        filt = re.compile(sys.argv[sys.argv.index("--filter") + 1])
        args = [a for a in args if a != filt.pattern]
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(lambda: collections.defaultdict(int))
    for d in args:
        for k, c in load(d).items():
            for n, v in c.items():
                tot[k][n] += v
                cnt[k][n] += 1
    print(f"{'kernel':52s} {'grid':>9s} {'mfma':>5s} {'wait':>5s} {'stall':>5s} {'ldsst':>5s} {'valu/mf':>7s} "
          f"{'lds/mf':>6s} {'vmem/mf':>7s} {'salu/mf':>7s} {'bank':>5s}")
    for k in sorted(tot, key=lambda k: -tot[k].get("SQ_VALU_MFMA_BUSY_CYCLES", 0)):
        if filt and not filt.search(k[0]):
            continue
        c = {n: v / cnt[k][n] if n in ("GRBM_GUI_ACTIVE", "SQ_WAVES") else v for n, v in tot[k].items()}
        g = c.get("GRBM_GUI_ACTIVE", 0) / 8
        mb = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)
        nm = mb / 32 if mb else 0
        wc = c.get("SQ_WAVE_CYCLES", 0)

        def f(x, den, w=5, p=2):
            return f"{x / den:{w}.{p}f}" if den and x is not None else " " * (w - 1) + "-"
        print(f"{k[0]:52s} {k[1]:>9s} {f(mb, 1024 * g)} {f(c.get('SQ_WAIT_ANY'), wc)} "
              f"{f(c.get('SQ_WAIT_INST_ANY'), wc)} {f(c.get('SQ_WAIT_INST_LDS'), wc)} "
              f"{f(c.get('SQ_INSTS_VALU'), nm, 7)} {f(c.get('SQ_INSTS_LDS'), nm, 6)} {f(c.get('SQ_INSTS_VMEM'), nm, 7)} "
              f"{f(c.get('SQ_INSTS_SALU'), nm, 7)} {f(c.get('SQ_LDS_BANK_CONFLICT'), c.get('SQ_ACTIVE_INST_LDS'))}")


if __name__ == "__main__":
    main()
