set -o pipefail
for wl in c3 c2; do for v in base rs64 rs32; do
  bash tools/kstats.sh ${v}_$wl L5DH_LIB=$(pwd)/linkerd_amd/lib_ab/lib$v.so --workload $wl || exit 1
done; done
