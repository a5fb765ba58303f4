set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/ab_nt
mkdir -p $OUT
for i in 1 2 3; do
  for v in A B C; do
    RSG_LIB_PATH=$R/rustfs_amd/ab/$v.so timeout -k 10 120 python -u bench.py --no-extras --no-cpu-baseline --no-rs12 --no-config-extras > $OUT/$v$i.json 2> $OUT/$v$i.err || exit 1
    python -c "import json; d=json.loads(open('$OUT/$v$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v$i', r['kernel_ms_avg'], r['frac'])"
  done
done
