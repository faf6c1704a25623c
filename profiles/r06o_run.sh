set -o pipefail
# first-hop what-if kernel: parity tests, then the what-if batch
D=gpurun_out/r06o; mkdir -p $D
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_whatif_firsthop_gpu.py tests/test_whatif_repair_gpu.py > $D/gpu_tests.log 2>&1 || { tail -60 $D/gpu_tests.log; exit 3; }
tail -3 $D/gpu_tests.log
timeout -k 10 300 python profiles/whatif_probe.py 5 > $D/wi.json 2> $D/wi.err || { tail -20 $D/wi.err; exit 4; }
OPENR_SPF_WHATIF_FIRSTHOP=0 timeout -k 10 300 python profiles/whatif_probe.py 5 > $D/wi_fh0.json 2> $D/wi_fh0.err || { tail -20 $D/wi_fh0.err; exit 5; }
python3 - <<PY
import json
for f in ("wi", "wi_fh0"):
    d = json.loads(open("$D/%s.json" % f).read().strip().splitlines()[-1])
    print(f, d.get("ms"), d.get("device_ms"), d.get("value"), d.get("parity_check"), d.get("kernels_launched"))
PY
