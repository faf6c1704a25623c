set -o pipefail
D=gpurun_out/r03z; mkdir -p $D
timeout -k 10 300 python profiles/scaling_probe.py > $D/scaling_probe.json 2> $D/probe.err || exit 5
cat $D/scaling_probe.json | python -c "import json,sys; d=json.load(sys.stdin); [print(k, v['sources'], v['kernel'], v['ms'], v['stage_ms']) for k,v in d.items()]"
