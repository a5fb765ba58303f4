# Sourced by the A/B scripts that choose kernels through RSG_* environment
# variables: since ABI 6 only a measurement build reads them (the shipped
# library ignores the environment).  Build it here first, on the CPU:
#   make -j8 -C rustfs_amd/csrc MEASURE=1      # -> rustfs_amd/measure/librsgpu.so
_R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)}
export RSG_LIB_PATH=$_R/rustfs_amd/measure/librsgpu.so
if [ ! -f "$RSG_LIB_PATH" ]; then
  echo "measure_env.sh: $RSG_LIB_PATH missing: make -C rustfs_amd/csrc MEASURE=1 first" >&2
  exit 2
fi
