# GPU A/B of variant libraries on 4:4:4 q90 and true 4:2:2 q75 (parity-checked bench runs).
# Usage (GPU box): bash tools/g_ab.sh reps variant...
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
R=$1; shift
REPS=$R bash tools/gpu_libs_bench.sh default "$@" || exit 1
BENCH_ARGS="--subsample --sample-ratio 1 --quality 75" REPS=$R bash tools/gpu_libs_bench.sh default "$@"
