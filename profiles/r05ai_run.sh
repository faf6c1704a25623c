set -o pipefail
# link flap after edge-balanced host blocks + fused passes
D=gpurun_out/r05ai; mkdir -p $D
R=$(pwd)
timeout -k 10 400 python -u -m pytest tests/test_graph_update_gpu.py tests/test_engine_parity_gpu.py -k "update or link_flap or selective_memo or incremental" -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -30 $D/gpu_tests.log; exit 2; }
tail -1 $D/gpu_tests.log
OPENR_SPF_CREATE_TIMING=1 OPENR_LS_SPLICE_TIMING=1 timeout -k 10 300 python3 profiles/linkflap_probe.py > $D/linkflap.json 2> $D/linkflap.err || { tail -5 $D/linkflap.err; exit 5; }
python3 -c "import json; d=json.load(open('$D/linkflap.json')); print({k: d.get(k) for k in ('ms_median','update_ms_median','build_ms_median','parity_check','per_build_us')})"
tail -22 $D/linkflap.err
