set -o pipefail
# no swar launch on graphs of <= 254 nodes: grid A/B, full GPU suite, smoke
D=gpurun_out/r06bg; mkdir -p $D
OPENR_NL_SWAR_SKIP=0 timeout -k 10 200 python3 profiles/grid_probe.py --iters 300 > $D/grid_off.json 2>/dev/null || exit 3
timeout -k 10 200 python3 profiles/grid_probe.py --iters 300 > $D/grid_on.json 2>/dev/null || exit 4
python3 -c "
import json
for t in ('off','on'):
    j=json.load(open('$D/grid_%s.json'%t)); e=j['engine']['per_build_us']
    print(t, j['engine']['ms_median'], e.get('decision.spf_batch_us'), e.get('decision.spf_device_us'), 'oracle', j['cpu_oracle']['ms_median'])"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $D/gpu_tests.log 2>&1 || { tail -40 $D/gpu_tests.log; exit 5; }
tail -1 $D/gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 6; }
tail -1 $D/smoke.log
