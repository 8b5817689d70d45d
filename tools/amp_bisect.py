"""Run the AMP BEVNet float64-reference test under flag combinations (epilogue BN statistics, fp16 projection
panels) and print the worst error ratios of each.  (GPU box)"""
import os
import sys
import traceback

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
import conftest  # noqa: E402,F401  (paths)
import test_train_amp_gpu as t  # noqa: E402
from models import model_wrapper  # noqa: E402
from models.encoders import trunk_grad  # noqa: E402

for ep, hp in ((True, True), (False, True), (True, False), (False, False)):
    trunk_grad.EPILOGUE_BN_STATS, model_wrapper.AMP_FWD_HALF_PANELS = ep, hp
    try:
        t.test_bevnet_r50_training_step_vs_float64_reference(True)
        print(f"epilogue_stats={ep} fwd_half_panels={hp}: PASS", flush=True)
    except AssertionError as e:
        print(f"epilogue_stats={ep} fwd_half_panels={hp}: FAIL {e}", flush=True)
    except Exception:
        traceback.print_exc()
