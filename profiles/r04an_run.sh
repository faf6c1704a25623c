set -o pipefail
# round 4: the deep-graph rerun test (both MS-BFS flag words)
D=gpurun_out/r04an; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_abi_gpu.py -m gpu -x -q -k "deep" --timeout 120 --timeout-method thread > $D/deep.log 2>&1 || { tail -15 $D/deep.log; exit 2; }
tail -1 $D/deep.log
