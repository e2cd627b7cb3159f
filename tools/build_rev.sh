#!/bin/bash
# Build libkfmi from git revision REV into sensorfusion-kalmanfilter_amd/kfmi/libkfmi_NAME.so
# (for in-session A/B on the GPU box: tools/ab_inproc.py --arms sensorfusion-kalmanfilter_amd/kfmi/libkfmi_NAME.so,default;
# a build from another revision carries another source hash, so loading it as KFMI_LIB needs
# KFMI_ALLOW_FOREIGN_LIB=1).
set -eu
REV=$1; NAME=$2
ROOT=$(git rev-parse --show-toplevel)
TMP=$(mktemp -d)
git -C "$ROOT" archive "$REV" sensorfusion-kalmanfilter_amd include | tar -x -C "$TMP"
make -C "$TMP/sensorfusion-kalmanfilter_amd" -j8 OUT="$ROOT/sensorfusion-kalmanfilter_amd/kfmi/libkfmi_$NAME.so" >/dev/null
rm -rf "$TMP"
echo "built libkfmi_$NAME.so from $REV"
