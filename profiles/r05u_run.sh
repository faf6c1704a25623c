set -o pipefail
# round 5: cooperative MS-BFS with write-through publishes (no release
# fence) + parity; link flap without the shared_ptr table copy + flap tests
D=gpurun_out/r05u; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_msbfs_coop_gpu.py tests/test_graph_update_gpu.py tests/test_engine_parity_gpu.py -k "coop or update or link_flap or selective_memo or incremental" -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -30 $D/gpu_tests.log; exit 3; }
tail -1 $D/gpu_tests.log
timeout -k 10 300 python3 profiles/scaling_probe.py > $D/scaling_probe.json 2> $D/scaling_probe.err || { tail -5 $D/scaling_probe.err; exit 5; }
python3 -c "
import json; d=json.load(open('$D/scaling_probe.json'))
for k,v in d.items(): print(k, v['sources'], v['ms'], v['stage_ms'])"
OPENR_MS_NOREC=1 timeout -k 10 300 python3 profiles/scaling_probe.py > $D/scaling_norec.json 2> $D/scaling_norec.err || { tail -5 $D/scaling_norec.err; exit 5; }
python3 -c "
import json; d=json.load(open('$D/scaling_norec.json'))
for k,v in d.items(): print('norec', k, v['sources'], v['ms'], v['stage_ms'])"
OPENR_SPF_CREATE_TIMING=1 timeout -k 10 300 python3 profiles/linkflap_probe.py > $D/linkflap.json 2> $D/linkflap.err || { tail -5 $D/linkflap.err; exit 4; }
python3 -c "import json; d=json.load(open('$D/linkflap.json')); print({k: d.get(k) for k in ('ms_median','update_ms_median','build_ms_median','parity_check','per_build_us')})"
