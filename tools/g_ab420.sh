# GPU A/B of variant libraries on true 4:2:0 q75 only.  Usage (GPU box): bash tools/g_ab420.sh reps variant...
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
R=$1; shift
BENCH_ARGS="--subsample --sample-ratio 2 --quality 75" REPS=$R bash tools/gpu_libs_bench.sh default "$@"
