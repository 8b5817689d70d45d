"""Per-layer conv timing from a rocprofv3 kernel trace of bench.py (ResNet-50, 7 x 1080x1920)."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/prof_conv/run_kernel_trace.csv'
rows = [r for r in csv.DictReader(open(path))
        if 'k_conv' in r['Kernel_Name'] or 'maxpool' in r['Kernel_Name'] or 'warp' in r['Kernel_Name']]
N = 7
L = []


def conv(name, ci, co, k, s, h, w):
    ho = (h + 2 * (k // 2) - k) // s + 1
    wo = (w + 2 * (k // 2) - k) // s + 1
    L.append((name, 2 * N * ho * wo * co * ci * k * k, ci, co, k, s, ho, wo))
    return ho, wo


h, w = conv('stem', 3, 64, 7, 2, 1080, 1920)
L.append(('maxpool', 0, 0, 0, 0, 0, 0, 0))
h, w = (h + 2 - 3) // 2 + 1, (w + 2 - 3) // 2 + 1
inp = 64
for bi in range(3):
    if bi == 0:
        conv('l1.0.ds', 64, 256, 1, 1, h, w)
    conv(f'l1.{bi}.c1', inp, 64, 1, 1, h, w)
    conv(f'l1.{bi}.c2', 64, 64, 3, 1, h, w)
    conv(f'l1.{bi}.c3', 64, 256, 1, 1, h, w)
    inp = 256
for bi in range(4):
    if bi == 0:
        conv('l2.0.ds', 256, 512, 1, 2, h, w)
        conv('l2.0.c1', 256, 128, 1, 1, h, w)
        h2, w2 = conv('l2.0.c2', 128, 128, 3, 2, h, w)
        conv('l2.0.c3', 128, 512, 1, 1, h2, w2)
        h, w = h2, w2
    else:
        conv(f'l2.{bi}.c1', 512, 128, 1, 1, h, w)
        conv(f'l2.{bi}.c2', 128, 128, 3, 1, h, w)
        conv(f'l2.{bi}.c3', 128, 512, 1, 1, h, w)
conv('proj', 512, 64, 1, 1, h, w)
L.append(('warp', 0, 0, 0, 0, 0, 0, 0))
seq = rows[-len(L):]
tot = 0
flops = 0
for (name, fl, ci, co, k, s, ho, wo), r in zip(L, seq):
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    tot += d
    flops += fl
    tf = fl / d / 1e6 if fl else 0
    print(f"{name:9s} {r['Kernel_Name'][:34]:34s} {d:8.1f}us M={N*ho*wo:8d} K={ci*k*k:5d} N={co:4d} {tf:6.1f} TF")
print(f'total {tot:.1f} us, conv {flops/1e12:.3f} TFLOP')
