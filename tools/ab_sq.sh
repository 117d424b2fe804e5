# SQ counters per variant: tools/ab_sq.sh dir v1 v2 ...
set -o pipefail
d=$1; shift
for v in "$@"; do
  cp $d/libccsc_$v.so ccsc_code_iccv2017_amd/libccsc.so
  bash tools/sq_profile.sh $v || exit 1
done
