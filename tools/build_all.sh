#!/bin/bash
# Build libfaasbal.so + the diagnostic stamps variant + the oracle; fail loudly.
set -e
cd "$(dirname "$0")/.."
python - <<'PY'
import sys, os
sys.path.insert(0, 'distributed-faas_amd')
from faasbal.build import build_lib, HERE
build_lib()
build_lib(out=os.path.join(HERE, 'libfaasbal_stamps.so'), defines=['FAASBAL_STAMPS'])
PY
make -s -C oracle
echo BUILD_OK
