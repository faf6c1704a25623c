set -o pipefail
# graph preparation on the device (derive + sliced-ELL kernels), edge-balanced
# host blocks, pool spin: full GPU suite, then the link-flap probe
D=gpurun_out/r05ak; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -30 $D/gpu_tests.log; exit 3; }
tail -1 $D/gpu_tests.log
OPENR_SPF_CREATE_TIMING=1 OPENR_LS_SPLICE_TIMING=1 timeout -k 10 300 python3 profiles/linkflap_probe.py > $D/linkflap.json 2> $D/linkflap.err || { tail -5 $D/linkflap.err; exit 5; }
python3 -c "import json; d=json.load(open('$D/linkflap.json')); print({k: d.get(k) for k in ('ms_median','update_ms_median','build_ms_median','parity_check','per_build_us')})"
tail -16 $D/linkflap.err
