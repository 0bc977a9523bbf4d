set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
A="default tools/ubench/libablate_1.so tools/ubench/libablate_2.so tools/ubench/libablate_8.so tools/ubench/libablate_16.so tools/ubench/libablate_256.so movement"
timeout -k 10 100 python tools/ramp.py --launches 300 --every 50 > gpurun_out/ramp2.log 2>&1
timeout -k 10 300 python tools/lib_ab.py --rounds 10 --b2b 4 $A > gpurun_out/abl_b2b.log 2>&1
cat gpurun_out/ramp2.log gpurun_out/abl_b2b.log | grep -v amdgpu.ids
