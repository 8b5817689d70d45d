"""A/B helper: run a script with bev_native loading another build of the library.
usage: python tools/with_lib.py <libbev.so> <script.py> [args...]"""
import os
import runpy
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "vision-based-spatio-temporal-analysis_amd"))
import bev_native  # noqa: E402

bev_native.LIB_PATH = os.path.abspath(sys.argv[1])
script = sys.argv[2]
sys.argv = sys.argv[2:]
sys.path.insert(0, os.path.dirname(os.path.abspath(script)))
runpy.run_path(script, run_name="__main__")
