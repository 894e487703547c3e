#!/bin/bash
# Round-3 probe 7: the weights' T image as streaming stores (A/B against moments-only).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
AB_TAG=_ntp bash tools/ablib.sh sac-td3-td7_amd/lib/librle.so sac-td3-td7_amd/lib/librle_ntp.so 3 3000 || exit 1
