set -o pipefail
# what-if: source-link failures in their own BFS kernel (uniform areas)
D=gpurun_out/r05av; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_whatif_repair_gpu.py tests/test_abi_gpu.py tests/test_config_sized_gpu.py tests/test_golden.py -k "whatif or repair or screen or config5" -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -30 $D/gpu_tests.log; exit 2; }
tail -1 $D/gpu_tests.log
timeout -k 10 300 python3 profiles/whatif_probe.py 3 > $D/probe.json 2> $D/probe.err || { tail -5 $D/probe.err; exit 3; }
python3 -c "import json; d=json.load(open('$D/probe.json')); print({k: d.get(k) for k in ('ms','device_ms','value','screened_queries','parity_check')})"
R=$(pwd); cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $R/$D/trace -o run --output-format csv -- python3 $R/profiles/whatif_probe.py 3 > $R/$D/trace.json 2>&1 || exit 4
cd $R
head -12 $(find $D/trace -name "*kernel_stats.csv" | head -1)
