# A/B of the forward's tie strategies on the bench step (tools/lib_ab.py, 3 launches back to back per sample):
# default, the variants in tools/ubench/libvar_*.so, and the movement ceiling, over input kind x quality x adaptive.
set -e
mkdir -p gpurun_out
L="default $(ls tools/ubench/libvar_*.so | tr '\n' ' ') movement"
while read -r k q a; do
  [ -z "$k" ] && continue
  timeout -k 10 200 python -u tools/lib_ab.py $L --b2b 3 --kind $k --quality $q --adaptive $a > gpurun_out/ip_$k${q}a$a.log 2>&1
done <<< "${CASES:-uniform 50 0
extreme 10 0
uniform 100 0
smooth 50 0
uniform 90 0}"
