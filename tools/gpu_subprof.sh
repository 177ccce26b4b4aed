set -u
cd $GRAFT_REPO_ROOT; OUT=$GRAFT_REPO_ROOT/gpurun_out/subprof; mkdir -p $OUT; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
cd /tmp
JPGX_LIB=$R/jpeg-encoder-and-decoder_amd/lib/libjpgx_alt.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tp -o run -- python $R/bench.py --subsample --sample-ratio 1 --quality 75 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/tp.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/fu -o run -- python $R/bench.py --subsample --sample-ratio 1 --quality 75 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/fu.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/pm -o run -- python $R/bench.py --subsample --sample-ratio 1 --quality 75 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/pm.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmx -o run -- python $R/bench.py --kernel xform --steps 5 --warmup 2 --no-cpu-baseline > $OUT/pmx.log 2>&1 || exit 1
find $OUT -name "*kernel_stats.csv" | while read f; do echo "== $f"; cut -d, -f1-4 "$f" | head -6; done
