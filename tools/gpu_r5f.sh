set -u
mkdir -p gpurun_out/r5f
timeout -k 10 120 python tools/diag_rate.py 20 0 > gpurun_out/r5f/product.txt 2>&1 || exit $?
for v in bgd bgl bl0; do JPGX_LIB=$PWD/jpeg-encoder-and-decoder_amd/lib/variants/libjpgx_$v.so timeout -k 10 120 python tools/diag_rate.py 20 0 > gpurun_out/r5f/$v.txt 2>&1 || exit $?; done
grep -v amdgpu.ids gpurun_out/r5f/*.txt
