#!/bin/bash
# r02ba: the other BASELINE configs on the final tree: config 1 (small-cycle
# latency), config 4 (64-node epoch-change cycle, dedup), config 5 (12.5 M
# mixed-size requests per GPU, block-balanced sharder).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02ba; mkdir -p $O
timeout -k 10 300 python -u bench.py --config 1 > $O/bench_config1.jsonl 2> $O/c1.err || { tail $O/c1.err; exit 1; }
timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 2 --cpu-seconds 3 > $O/bench_config4.jsonl 2> $O/c4.err || { tail $O/c4.err; exit 1; }
timeout -k 10 400 python -u bench.py --config 5 --steps 3 --warmup 1 --cpu-seconds 5 > $O/bench_config5.jsonl 2> $O/c5.err || { tail $O/c5.err; exit 1; }
for f in $O/bench_config4.jsonl $O/bench_config5.jsonl; do python3 -c "import json; d=json.loads(open('$f').readlines()[-1]); print('$f', '%.4g' % d['value'], round(d['ms_per_step'],3), 'frac', round(d['roofline']['frac'],4), 'check', d.get('self_check'), 'cpu', '%.4g' % (d.get('cpu_baseline') or {}).get('value', 0), d.get('host_phases_ms'))"; done
python3 -c "import json; d=json.loads(open('$O/bench_config1.jsonl').readlines()[-1]); print([(c['hash_requests'], round(c['hash_slices_us'],1), round(c['submit_wait_us'],1), round(c['cpu_1core_us'],1)) for c in d['cycles']])"
echo all done
