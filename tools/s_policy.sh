set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
L="tools/ubench/libpolicy_2.so tools/ubench/libpolicy_0.so tools/ubench/libpolicy_noflag_2.so tools/ubench/libpolicy_noflag_0.so movement:tools/ubench/libpolicy_2.so movement:tools/ubench/libpolicy_0.so"
timeout -k 10 200 python tools/lib_ab.py --rounds 8 --b2b 4 $L > gpurun_out/pol_both.log 2>&1
timeout -k 10 200 python tools/lib_ab.py --rounds 8 --b2b 4 --luma-only $L > gpurun_out/pol_luma.log 2>&1
timeout -k 10 200 python tools/lib_ab.py --rounds 8 --b2b 4 --chroma-only $L > gpurun_out/pol_chroma.log 2>&1
cat gpurun_out/pol_*.log | grep -v amdgpu.ids
