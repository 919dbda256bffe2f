#!/bin/bash
# r03n: rocprofv3 kernel trace + PMC passes of the driver's bench command
# (config 2), config 3 (fused plan) and config 2 overlapped cycles.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash profiles/profile.sh r03n_c2 || exit 1
bash profiles/profile.sh r03n_c3 --config 3 || exit 1
bash profiles/profile.sh r03n_c2ovl --pipeline overlap || exit 1
echo all done
