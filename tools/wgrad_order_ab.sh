#!/bin/bash
# Same-box A/B of the split-major conv weight-gradient tile order (tools/lab/wgrad_split_major.diff, built into
# clip-ebc_amd/lib/exp_wg/libebc_hip.so) against the in-tree library: decoder / ResNet parity tests on the
# variant, conv_bench and the bench step interleaved.
set -e
O=gpurun_out; mkdir -p $O; T=$O/r03t_wgrad_order.txt; : > $T
EXP=$PWD/clip-ebc_amd/lib/exp_wg/libebc_hip.so
timeout -k 10 300 env EBC_LIB_PATH=$EXP python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_shapes.py tests/test_gpu_resnet.py > $O/r03t_tests.log 2>&1
for r in 1 2 3; do for e in "EBC_X=0" "EBC_LIB_PATH=$EXP"; do
  echo "r$r ${e##*/lib/}: $(timeout -k 10 120 env $e python -u tools/conv_bench.py 2>&1 | tail -1)" >> $T
done; done
bash tools/env_ab.sh r03t "--steps 30 --warmup 10" "EBC_X=0" "EBC_LIB_PATH=$EXP"
