set -e
for cfg in 2 3; do for pl in none fused; do
timeout -k 10 120 python bench.py --config $cfg --pipeline $pl --cpu-seconds 0 --no-pcie > gpurun_out/b_${cfg}_${pl}.json 2>/dev/null
done; done
