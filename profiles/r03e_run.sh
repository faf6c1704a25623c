set -o pipefail
R=$(pwd)
OPENR_NL_SWAR=1 timeout -k 10 400 bash profiles/prof_fabric_sq.sh r03e_swar > gpurun_out/r03e_swar.log 2>&1 || exit 3
tail -4 gpurun_out/r03e_swar.log
OPENR_NL_SWAR=0 timeout -k 10 400 bash profiles/prof_fabric_sq.sh r03e_scalar > gpurun_out/r03e_scalar.log 2>&1 || exit 4
tail -4 gpurun_out/r03e_scalar.log
