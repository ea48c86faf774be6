#!/bin/bash
# usage: abbuild.sh TAG [extra flags]  -> build_ab/lib_TAG.so
TAG=$1; shift
cd /root/repo/open_spiel-1_amd/csrc
make -s -j8 OBJ=build_$TAG OUT=../../build_ab/lib_$TAG.so FLAGS="-O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -shared -Wall -Wno-unused-function -Wno-unused-variable $*" 2>&1 | grep -E "error" 
ls -la ../../build_ab/lib_$TAG.so | awk '{print $5, $9}'
