set -o pipefail
mkdir -p gpurun_out/ring1
B=tools/kbench/ring_variants
timeout -k 10 120 $B 2097152 256 6 > gpurun_out/ring1/s16m.txt 2>&1 \
&& timeout -k 10 120 $B 1048576 512 6 > gpurun_out/ring1/s8m.txt 2>&1 \
&& timeout -k 10 120 $B 524288 1024 6 > gpurun_out/ring1/s4m.txt 2>&1 \
&& timeout -k 10 120 $B 262144 2048 6 > gpurun_out/ring1/s2m.txt 2>&1 \
&& timeout -k 10 120 $B 131072 4096 6 > gpurun_out/ring1/s1m.txt 2>&1
