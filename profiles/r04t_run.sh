set -o pipefail
# round 4: inline address / interface-name strings in the thrift types (SmallString):
# + few-source plans (MS-BFS with helper rows below 32 sources; weighted few-source batches: helper rows on the LDS-row pass + spf_nh_rows_kernel):
# the whole GPU suite, then the RouteDb / KSP2 rebuild loops, link flaps, what-if
D=gpurun_out/r04t; mkdir -p $D
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1; rc=$?
tail -3 $D/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 profiles/route_db_probe.py 6 > $D/route_db_probe.json 2> $D/route_db_probe.err || exit 3
python3 - <<'PY'
import json
d=[json.loads(l) for l in open('gpurun_out/r04t/route_db_probe.json') if l.startswith('{')][-1]
for k in ('route_db_rebuild','ksp2_route_db'):
    v=d[k]; print(k, {x: v.get(x) for x in ('ms_median','build_ms_median','update_ms_median','release_ms_median','parity_check')})
    print('  ', v.get('per_build_us') or v.get('per_build'))
PY
timeout -k 10 300 python3 profiles/linkflap_probe.py > $D/linkflap.log 2>&1 || exit 4
grep '^{' $D/linkflap.log | cut -c1-400
timeout -k 10 300 python3 profiles/whatif_split_probe.py > $D/split.log 2>&1 || exit 5
grep '^{' $D/split.log
timeout -k 10 240 python3 profiles/whatif_probe.py 3 > $D/whatif.log 2>&1 || exit 6
grep '^{' $D/whatif.log | cut -c1-600
