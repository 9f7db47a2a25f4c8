#!/bin/bash
# Build lib/libsbo_base.so from HEAD (working-tree changes stashed meanwhile), then rebuild this tree.
set -e
cd "$(dirname "$0")/.."
git stash -q
(cd safe_bayesian_optimization_amd && make -s -j8 ARCH=gfx950 lib/libsbo.so && cp lib/libsbo.so lib/libsbo_base.so) || { git stash pop -q; exit 1; }
git stash pop -q
cd safe_bayesian_optimization_amd && make -s -j8 ARCH=gfx950
md5sum lib/libsbo.so lib/libsbo_base.so
