set -u
cd "${GRAFT_REPO_ROOT}"
timeout -k 10 300 python tools/exp/l3dbg.py || exit 1
bash tools/exp/ab_lib.sh ${1:-l3ab3} "--op l3fwd --packets 4194304" || exit 1
bash tools/exp/l3prof2.sh ${1:-l3ab3}_prof
