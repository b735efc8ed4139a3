#!/bin/bash
# Builds an experiment variant of libigx.so (A/B against the default build):
# the default build's objects are copied, the listed device parts (IGX_PART,
# see igx_device.hip's head: 0 host + small kernels, 1 k_extend, 2 k_finish,
# 3 trace / shade / shadow kernels) are rebuilt with the extra flags.
# usage: build_variant.sh NAME "EXTRA flags" [parts, default "0 1 2 3"]
# -> ignis-masterthesis_amd/libigx_NAME.so (IGX_LIB_PATH selects it at run time)
set -e
cd "$(dirname "$0")/../ignis-masterthesis_amd"
NAME=$1; EXTRA=$2; PARTS=${3:-"0 1 2 3"}
make -s -j8 >/dev/null  # the default build is current
rm -rf build_$NAME && cp -a build build_$NAME
for p in $PARTS; do rm -f build_$NAME/igx_device_p$p.o; done
make -s -j8 BUILD=build_$NAME LIB=libigx_$NAME.so EXTRA="$EXTRA" libigx_$NAME.so
ls -la libigx_$NAME.so
