# GPU A/B of variant libraries on true 4:2:2 q75 only.  Usage (GPU box): bash tools/g_ab422.sh reps variant...
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
R=$1; shift
BENCH_ARGS="--subsample --sample-ratio 1 --quality 75" REPS=$R bash tools/gpu_libs_bench.sh default "$@"
