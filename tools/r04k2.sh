#!/bin/bash
# Round-4 GPU pass k2: config-4 knob sweep after the fp32-beta post pass.
set -o pipefail
timeout -k 10 900 bash tools/dl_tune.sh 2 - post_pairs=1 post_pairs=4 dl_lane=1 dl_split=1 side_priority=1 || exit 1
