"""pytest entry for tools/with_lib.py (a variant library's parity run):

    python tools/with_lib.py tools/_ab/libbev_ck32o4.so tools/run_pytest.py tests/test_warp_gpu.py -x -q
"""
import sys

import pytest

sys.exit(pytest.main(sys.argv[1:]))
