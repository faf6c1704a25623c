set -o pipefail
# what-if repair on the global-memory SSSP (OPENR_SPF_WHATIF_GMEM=1) with 2 / 4
# workgroups per CU, against the LDS plan (2 per CU, LDS-bound)
D=gpurun_out/r06at; mkdir -p $D
for cfg in "lds:0:2" "gmem2:1:2" "gmem4:1:4" "lds_b:0:2" "gmem4_b:1:4"; do
  IFS=: read tag g p <<< "$cfg"
  OPENR_SPF_WHATIF_GMEM=$g OPENR_SPF_GMEM_PERCU=$p timeout -k 10 200 python3 profiles/whatif_probe.py 8 > $D/wi_$tag.json 2> $D/wi_$tag.err || { tail -5 $D/wi_$tag.err; exit 3; }
  python3 -c "import json; j=json.load(open('$D/wi_$tag.json')); print('$tag', j.get('ms'), j.get('device_ms'), j.get('parity_check'))"
done
