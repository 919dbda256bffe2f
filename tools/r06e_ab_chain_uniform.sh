set -e
mkdir -p gpurun_out/r06e
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "uniform_lists or pipeline_device_full_size or pipeline_overlap or irregular" > gpurun_out/r06e/tests.log 2>&1
for i in 1 2 3; do
  for u in 1 0; do
    MIRSHA_AB=1 MIRSHA_CHAIN_UNIFORM=$u timeout -k 10 120 python -u bench.py --steps 50 --warmup 20 --cpu-seconds 0 --no-pcie --no-config3-leg --no-overlap-extra > gpurun_out/r06e/ab_u${u}_$i.jsonl 2>/dev/null
  done
done
echo done
