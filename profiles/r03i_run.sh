set -o pipefail
D=gpurun_out/r03i; mkdir -p $D
Q="--no-cpu-baseline --no-route-db --no-wan --no-whatif --no-repair --steps 20 --warmup 3"
for v in "64 0" "64 1" "32 0"; do set -- $v
  OPENR_SPF_MSBFS=$1 OPENR_NL_XCD=$2 timeout -k 10 200 python bench.py $Q > $D/fab_m$1x$2.json 2> $D/fab_m$1x$2.err || exit 7
  python -c "import json;d=json.load(open('$D/fab_m$1x$2.json'));print('msbfs',$1,'xcd',$2,d['ms_per_step'],d.get('kernels'),d.get('parity_spot_check'))"
done
