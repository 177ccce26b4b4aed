# GPU: parity suites (4:4:4 + subsampling) then an interleaved A/B of variant libraries on 4:4:4 q90
# and true 4:2:2 q75.  Usage (GPU box): bash tools/g_t_ab.sh reps variant...
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_subsample.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_ab.log 2>&1; rc=$?
tail -3 gpurun_out/t_ab.log; grep -E "^FAILED|Error|assert" gpurun_out/t_ab.log | head -20
[ $rc -eq 0 ] || exit $rc
bash tools/g_ab.sh "$@"
