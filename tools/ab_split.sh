timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/t.log 2>&1; tail -2 gpurun_out/t.log
. "$(dirname "$0")/measure_env.sh"  # RSG_* knobs: the measurement build (ABI 6)
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras"
for kk in 16 12; do
 for sp in 1 0; do
  RSG_SPLIT=$sp timeout -k 10 300 $B --k $kk --m 4 > gpurun_out/s_${kk}_${sp}.json 2>/dev/null || exit 1
  echo "k=$kk split=$sp $(python -c "import json; d=json.load(open('gpurun_out/s_${kk}_${sp}.json')); print(d['value'], d['roofline']['kernel_ms_avg'], d['roofline']['frac'])")"
 done
done
