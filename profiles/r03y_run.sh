set -o pipefail
D=gpurun_out/r03y; mkdir -p $D
B="bench.py --no-cpu-baseline --no-route-db --no-whatif --no-wan --steps 30 --warmup 5"
for x in 0 1 0 1; do
  OPENR_MS_WREC=$x timeout -k 10 200 python $B > $D/wrec$x.json 2>> $D/err.log || exit 5
  python -c "import json;d=json.load(open('$D/wrec$x.json'));print('wrec=$x', d['ms_per_step'], d['kernels'], d['parity_spot_check'])"
done
