#!/bin/bash
# Build an A/B variant of librmc + raftmc in raft-tlaplus_amd/<dir> that differs
# from raft-tlaplus_amd/build only in rmc_kernels.o (compiled with EXTRA flags):
# the host objects are copied from build/ (make build first).
#   tools/variant.sh build_legacy "-DRMC_FP_LEGACY"
set -e
cd "$(dirname "$0")/../raft-tlaplus_amd"
D=$1
FLAGS=$2
mkdir -p $D
for o in rmc_engine rmc_host rmc_sharded rmc_simulate rmc_cpu; do cp -p build/$o.o $D/; done
rm -f $D/rmc_kernels.o
make OUT=$D EXTRA="$FLAGS" $D/librmc.so $D/raftmc
