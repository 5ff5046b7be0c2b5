#!/bin/bash
# Round-4 measurement session: GPU suite + smoke + bench under rocprofv3 (tools/sessions/r04_session.sh),
# then the counter session on the timed kernels.  bash tools/sessions/r04_final.sh <tag>  (on the box)
set -o pipefail
T=${1:-final}
bash tools/sessions/r04_session.sh $T || exit 1
NO_PMC= bash tools/sessions/r04_counters.sh c_$T || exit 1
