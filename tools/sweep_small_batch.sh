set -e
. "$(dirname "$0")/measure_env.sh"  # RSG_* knobs: the measurement build (ABI 6)
mkdir -p gpurun_out/small
for kib in 2048 4096 8192 16384; do
  bytes=$((kib*1024)); n4=$(( (4*1024*1024*1024)/bytes ))
  for f in 1 0; do
    RSG_FUSED=$f timeout -k 10 300 python bench.py --stripe-bytes $bytes --batch $n4 --digests --steps 10 --warmup 2 --no-extras --no-cpu-baseline > gpurun_out/small/s${kib}k_f$f.json
    echo "$kib KiB n=$n4 fused=$f $(tail -1 gpurun_out/small/s${kib}k_f$f.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms_avg"])')"
  done
done
