set -o pipefail
bash profiles/calib/run_calib.sh && bash profiles/prof_fabric.sh r03q
