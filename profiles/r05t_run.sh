set -o pipefail
# round 5: per-rank probe with the MS-BFS row stores off (OPENR_MS_NOREC=1,
# measurement: does the cooperative split pay once the scattered level-row
# stores are gone?); link-flap weight scan after the false-sharing fix
D=gpurun_out/r05t; mkdir -p $D
OPENR_MS_NOREC=1 timeout -k 10 300 python3 profiles/scaling_probe.py > $D/scaling_norec.json 2> $D/scaling_norec.err || { tail -5 $D/scaling_norec.err; exit 5; }
python3 -c "
import json; d=json.load(open('$D/scaling_norec.json'))
for k,v in d.items(): print('norec', k, v['sources'], v['ms'], v['stage_ms'])"
for P in 2 4; do
OPENR_MS_COOP_P=$P timeout -k 10 300 python3 profiles/scaling_probe.py > $D/scaling_p$P.json 2> $D/scaling_p$P.err || { tail -5 $D/scaling_p$P.err; exit 5; }
python3 -c "
import json; d=json.load(open('$D/scaling_p$P.json'))
for k,v in d.items():
  if 'coop1' in k: print('P<=$P', k, v['sources'], v['ms'], v['stage_ms'])"
done
OPENR_SPF_CREATE_TIMING=1 timeout -k 10 300 python3 profiles/linkflap_probe.py > $D/linkflap.json 2> $D/linkflap.err || { tail -5 $D/linkflap.err; exit 4; }
python3 -c "import json; d=json.load(open('$D/linkflap.json')); print({k: d.get(k) for k in ('ms_median','update_ms_median','build_ms_median','parity_check','per_build_us')})"
grep "spf_graph_update" $D/linkflap.err | tail -13
