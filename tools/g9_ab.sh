#!/bin/bash
# g9 (k_lsearch<Go>, 65536 x 256) traffic attribution: per build tag the g9
# line and FETCH_SIZE / WRITE_SIZE passes.  Tags: default, nomt (OS_LS_AB=1),
# nolog (OS_LS_AB=2), none (OS_LS_AB=3); A/B libs built by tools/abbuild.sh.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/g9ab
for tag in "$@"; do
  mkdir -p gpurun_out/g9ab/$tag
  OS_AMD_LIB=$R/build_ab/lib_$tag.so timeout -k 10 300 python3 -u bench.py --config g9 --layout lane --steps 2 --warmup 1 \
    --no-cpu-baseline --parity-roots 0 > gpurun_out/g9ab/$tag/bench.json 2> gpurun_out/g9ab/$tag/bench.err || exit 1
  cd /tmp && export TMPDIR=/tmp
  i=0
  for c in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    OS_AMD_LIB=$R/build_ab/lib_$tag.so timeout -k 10 200 rocprofv3 --kernel-trace --pmc $c \
      -d "$R/gpurun_out/g9ab/$tag/p$i" -o run --output-format csv -- \
      python3 "$R/bench.py" --config g9 --layout lane --steps 1 --warmup 1 --no-cpu-baseline --parity-roots 0 \
      > "$R/gpurun_out/g9ab/$tag/p$i.log" 2>&1 || exit 1
  done
  cd "$R"
  python3 -c "import json;d=json.load(open('gpurun_out/g9ab/$tag/bench.json'));print('$tag', d['value'], d['ms_per_step'])"
done
echo g9ab-done
