set -o pipefail
# round 6: small-K what-if patch (parity, A/B, stats, trace) + where the v2
# pass's time goes (measurement modes)
bash profiles/r06f_run.sh || exit $?
bash profiles/r06e_run.sh || exit $?
