# Round 5 pass b: fused-warp ablation timings on the current kernel, and the new parity tests (4K camera-shard
# encoder, full-geometry K3 AMP step, CONV_H16_KERNEL=1 under autocast).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
ROUNDS=4 timeout -k 10 300 python -u tools/warp_ablate.py 0 1 2 4 8 16 14 24 30 31 > $O/ablate.txt 2>&1 || exit $?
timeout -k 10 1500 python -u -m pytest -x -v -s -p no:cacheprovider --timeout 1300 --timeout-method thread \
  "tests/test_train_amp_gpu.py::test_bottleneck_h16_under_kernel_knob_1" \
  "tests/test_backbone_gpu.py::test_resnet50_encoder_4k_camera_shard_geometry" \
  "tests/test_train_amp_gpu.py::test_bevnet_r50_amp_step_full_geometry" > $O/new_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/new_tests.log; exit $rc
