# round 4, call P: the GPU suite (incl. the host_multi child test) and the default bench
set -o pipefail
bash tools/verify_round.sh r04p || exit 1
echo ok
