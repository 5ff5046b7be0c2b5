#!/bin/bash
# Round-5 A/B of one bench model leg (default deepfm): the current library against a variant library,
# alternating, twice; a variant of the form NAME=VALUE is the current library under that environment
# setting instead.  Usage (on the box): bash tools/sessions/r05_ab_model.sh <tag> <variant.so|VAR=v> [model]
set -o pipefail
T=${1:-abm}; V=$2; M=${3:-deepfm}; O=gpurun_out/r05/$T; mkdir -p $O; export TMPDIR=/tmp
CUR=$PWD/implementation-of-rank-algorithm-for-mainstream-recommender-systems_amd/rankops/librankops.so
run() {  # <name> <lib> [VAR=value]
  local n=$1 lib=$2 ev=${3:-RANKOPS_AB_NONE=1}
  env RANKOPS_LIB=$lib $ev timeout -k 10 200 python bench.py --no-cpu --no-loader --no-train --no-sharded --models $M > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -5 $O/$n.err; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); m=d['models']['$M']; print('$n', round(m['samples_per_s']/1e6,2), 'M step', m['ms_per_step'], 'kernel', m.get('roofline', {}).get('avg_launch_ms'))"
}
for i in 1 2; do
  run cur_$i $CUR || exit 1
  case $V in
    *=*) run var_$i $CUR $V || exit 1 ;;
    *) run var_$i $PWD/$V || exit 1 ;;
  esac
done
echo ab done
