#!/bin/bash
# Round-4 combined GPU session: the GPU test suite on the product library, the golden-frame
# hazard diagnostics (LOEXP-12 build without / with the chain keep-alive), the short-wave kernels
# against their variants (tools/kbench.py), and the skeleton's occupancy / MFMA sweep.
# Every step has its own time limit; a failure ends the script.  Usage: bash tools/gpu_r4_combo.sh OUT
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/$1"; mkdir -p "$OUT" gpurun_out/r4d
export TMPDIR=/tmp
V=jpeg-encoder-and-decoder_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread --maxfail=3 > "$OUT/gpu_tests.txt" 2>&1
rc=$?; tail -4 "$OUT/gpu_tests.txt"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for v in lx12 lx12kc; do
  JPGX_LIB=$PWD/$V/libjpgx_$v.so timeout -k 10 240 python tools/diag_golden.py 4 > gpurun_out/r4d/c_$v.txt 2>&1 || exit $?
  echo "== $v"; grep "rep" gpurun_out/r4d/c_$v.txt | cut -c1-60
done
KB_SUB=0 timeout -k 10 400 python tools/kbench.py 2 nokc w1c3 legacy l2w5 l3 c2 > "$OUT/kb444.txt" 2>&1 || exit $?
KB_SUB=1 timeout -k 10 300 python tools/kbench.py 2 l422 s422w4 > "$OUT/kb422.txt" 2>&1 || exit $?
KB_SUB=2 timeout -k 10 300 python tools/kbench.py 2 l420 s420w4 > "$OUT/kb420.txt" 2>&1 || exit $?
cat "$OUT/kb444.txt" "$OUT/kb422.txt" "$OUT/kb420.txt"
if [ "${SKEL:-0}" = "1" ]; then
  timeout -k 10 300 ./tools/membench3 r4c > "$OUT/skel_r4c.txt" 2>&1 || exit $?
  cut -c1-150 "$OUT/skel_r4c.txt"
fi
