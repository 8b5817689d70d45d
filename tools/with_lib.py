"""Run a tool script against a variant build of the library (A/B timing of a compile-time knob):

    python tools/with_lib.py tools/_ab/libbev_lines0.so tools/train_step_bench.py --bevnet --amp

Points bev_native.LIB_PATH at the given .so before the script runs (the script imports bev_native first through
sys.modules, so it loads the variant).  Timing only; the product always loads the in-tree library.
"""
import os
import runpy
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vision-based-spatio-temporal-analysis_amd"))
sys.path.insert(0, REPO)

import bev_native  # noqa: E402

bev_native.LIB_PATH = os.path.abspath(sys.argv[1])
script = sys.argv[2]
sys.argv = sys.argv[2:]
sys.path.insert(0, os.path.dirname(os.path.abspath(script)))
runpy.run_path(script, run_name="__main__")
