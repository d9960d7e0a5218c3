set -e
O=gpurun_out; mkdir -p $O; T=$O/r03t_wgrad_order.txt; : > $T
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_shapes.py tests/test_gpu_resnet.py > $O/r03t_tests.log 2>&1
for r in 1 2 3; do for e in 0 1; do
  echo "r$r EBC_WGRAD_ORDER=$e: $(timeout -k 10 120 env EBC_WGRAD_ORDER=$e python -u tools/conv_bench.py 2>&1 | tail -1)" >> $T
done; done
bash tools/env_ab.sh r03t "--steps 30 --warmup 10" "EBC_WGRAD_ORDER=0" "EBC_WGRAD_ORDER=1"
