set -o pipefail
D=gpurun_out/r03aa; mkdir -p $D
timeout -k 10 300 python bench.py --sharded --no-cpu-baseline --no-route-db --no-whatif --no-wan --steps 20 --warmup 3 > $D/sharded.json 2> $D/sharded.err || exit 5
python -c "import json;d=json.load(open('$D/sharded.json'));print(d['value'], d['ms_per_step'], d['config'], d.get('with_row_gather'), d['parity_spot_check'])"
