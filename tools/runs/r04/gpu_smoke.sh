#!/bin/bash
cd "$GRAFT_REPO_ROOT" && timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2
