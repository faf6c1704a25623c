set -o pipefail
# round 5: v2 next-hop pass block order A/B (OPENR_NL_V2_ORDER 0 / 1 / 2) and
# the FETCH_SIZE pass of each order
D=gpurun_out/r05f; mkdir -p $D
R=$(pwd)
B="bench.py --no-cpu-baseline --no-route-db --no-whatif --no-wan --steps 20 --warmup 3"
for i in 1 2; do
for o in 0 1 2; do
OPENR_NL_V2_ORDER=$o timeout -k 10 300 python3 $B > $D/fabric.o$o.$i.json 2> $D/fabric.o$o.$i.err || { tail -5 $D/fabric.o$o.$i.err; exit 2; }
python3 -c "import json,sys; d=json.load(open('$D/fabric.o$o.$i.json')); print('order=$o', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items()}, d.get('parity_spot_check'))"
done
done
cd /tmp && export TMPDIR=/tmp
for o in 0 2; do
OPENR_NL_V2_ORDER=$o timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -T -d $R/$D/pmc_o$o -o run --output-format csv -- \
  python3 $R/$B --steps 3 --warmup 1 > $R/$D/pmc_o$o.json 2> $R/$D/pmc_o$o.err || { tail -3 $R/$D/pmc_o$o.err; exit 3; }
done
cd $R
for o in 0 2; do python3 profiles/collect_pmc.py $D/pmc_o$o $D/pmc_o$o $D/pmc_o$o.traffic.json > /dev/null && python3 -c "import json;d=json.load(open('$D/pmc_o$o.traffic.json'))['kernels']['spf_nh_levels_v2_kernel'];print('order=$o', d)"; done
