set -o pipefail
D=gpurun_out/r03n; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_abi_gpu.py -x -q --timeout 200 --timeout-method thread -k "20k or msbfs or swar" > $D/gpu_tests.log 2>&1; rc=$?
tail -3 $D/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --num-sws 20000 --no-cpu-baseline --no-route-db --no-wan --no-whatif --no-repair > $D/fabric20k.json 2> $D/fabric20k.err || exit 5
python -c "import json;d=json.load(open('$D/fabric20k.json'));print(d['value'],d['ms_per_step'],d['config'],d.get('kernels'),d.get('parity_spot_check'))"
timeout -k 10 900 python bench.py --cpu-full --no-route-db --no-wan --no-whatif --no-repair > $D/cpu_full.json 2> $D/cpu_full.err || exit 6
python -c "import json;d=json.load(open('$D/cpu_full.json'));print(json.dumps(d.get('cpu_baseline'))[:3000])"
