set -o pipefail
# round 4: PMC passes over the LDS-row WAN kernel, then the fabric step profile (byte masks)
D=gpurun_out/r04f; mkdir -p $D
timeout -k 10 500 bash profiles/pmc_wan.sh r04f_wan 2048 base spf_dlds_kernel > $D/pmc_wan.log 2>&1 || exit 3
timeout -k 10 600 bash profiles/prof_fabric.sh r04f > $D/prof.log 2>&1 || exit 6
mkdir -p $D/prof && cp gpurun_out/prof_r04f/final/* $D/prof/
python -c "import json;d=json.load(open('$D/prof/trace_bench.json'));print(d['value'], d['ms_per_step'], d['roofline'])"
