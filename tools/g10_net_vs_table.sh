mkdir -p gpurun_out/g10
for L in 0 0,9 3,7 0,10 2; do
  for T in 1 0; do
    timeout -k 10 200 python -u tools/geom_engines.py 10,4 --get-lost $L --heal-lost 1,10 --tune RSG_DECODE_NET=$T > gpurun_out/g10/get_${L}_net$T.jsonl 2>> gpurun_out/g10/err.txt || exit 1
  done
done
echo done
