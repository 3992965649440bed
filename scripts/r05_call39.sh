#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
for v in 0 1 0 1; do SPG_HALVED_ENC=$v timeout -k 10 200 python scripts/micro/halved_rows.py || exit 1; done
