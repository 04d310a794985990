#!/bin/bash
# Round-4 profiles: the log-mel kernel (HIP-event line, kernel trace, PMC bytes), then the PMC
# passes and kernel traces of tools/probes/profile_r04.sh (its last step is the shipped cooperative
# launch under rocprofv3, whose exit status it records).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/probes/logmel_profile.sh || exit 1
bash tools/probes/profile_r04.sh
