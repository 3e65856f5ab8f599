set -o pipefail
cd $GRAFT_REPO_ROOT
export PROBE_B=131072,262144,524288
export PROBE_CFG=2:0,3:2048,3:3072,3:4096
for cfg in "base:libmgpu.so:4" "base1:libmgpu.so:1" "wpe3:libmgpu_wpe3.so:4" "wpe4:libmgpu_wpe4.so:4"; do
  IFS=: read tag lib wg <<< "$cfg"
  PROBE_TAG=$tag MGPU_LIB=$PWD/minotaur_amd/$lib MGPU_FBBT_WG=$wg timeout -k 10 200 python -u tools/fbbt_refill_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
done
