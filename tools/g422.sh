# GPU: parity of the MFMA kernels (4:4:4 parity suite + subsampling suite), then bench lines for
# 4:4:4 q90 and true 4:2:2 / 4:2:0 q75.  Usage (GPU box): bash tools/g422.sh [reps]
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_subsample.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t422.log 2>&1; rc=$?
tail -3 gpurun_out/t422.log; grep -E "^FAILED|Error|assert" gpurun_out/t422.log | head -20
[ $rc -eq 0 ] || exit $rc
for i in $(seq 1 ${1:-2}); do
  timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/b444_$i.json || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1], r['kernel'], r['kernel_ms'], r['frac'])" gpurun_out/b444_$i.json
  for sr in 1 2; do
    timeout -k 10 120 python bench.py --subsample --sample-ratio $sr --quality 75 --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/b42${sr}_$i.json || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1], r['kernel'], r['kernel_ms'], r['frac'])" gpurun_out/b42${sr}_$i.json
  done
done
