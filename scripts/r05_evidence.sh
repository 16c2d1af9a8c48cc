#!/bin/bash
# round 5 evidence run: default bench + rocprof step table + PMC (scripts/evidence.sh), then the
# preset / configs bench lines
set -o pipefail
bash scripts/evidence.sh r05b || exit 1
bash scripts/r05_presets.sh || exit 1
