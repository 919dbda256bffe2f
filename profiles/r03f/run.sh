#!/bin/bash
# r03f: split tiles in the fused launch: parity (split tiles, config 3 full
# size, fused irregular, overlap cycles, fail-closed), then config 3 bench
# (fused step + overlapped cycle) and the fused timeline.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03f; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "split or fused or full_size or overlap or watchdog" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie > $O/bench_c3.jsonl 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench_c3.jsonl').readlines()[-1]); r=d['roofline']; o=d.get('overlap_cycles') or {}
print('c3 step', round(d['ms_per_step'],4), 'kern', round(r['avg_launch_ms']*1e3,1), 'frac', round(r['frac'],4), 'check', d['self_check'], 'overlap', round(o.get('ms_per_step',0),4), round(o.get('frac',0),4))"
timeout -k 10 200 python -u tools/trace_fused.py 3 0 > $O/trace_c3.jsonl 2> $O/trace.err || { tail -20 $O/trace.err; exit 1; }
cut -c1-1500 $O/trace_c3.jsonl
timeout -k 10 200 python -u -m pytest tests/test_c_abi.py -x -q --timeout 120 --timeout-method thread > $O/pytest_c.log 2>&1 || { tail -30 $O/pytest_c.log; exit 1; }
tail -1 $O/pytest_c.log
timeout -k 10 200 tests/c/build/cgo_path 1048576 256 16 5 > $O/cgo_path.json 2>&1 || { cat $O/cgo_path.json; exit 1; }
cat $O/cgo_path.json
