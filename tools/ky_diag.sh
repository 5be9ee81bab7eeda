# The y-form pass taken apart: the normal build and three
# diagnostic builds (build/diagN, -DKT_KY_DIAG=N), each timed alone (HIP events,
# one lane) and counted in separate rocprofv3 --pmc passes.
set -e
O=$PWD/gpurun_out/kydiag; mkdir -p $O
export TMPDIR=/tmp
for v in normal diag1 diag2 diag3; do
  if [ $v = normal ]; then LIB=$PWD/krylov_robustness_amd/libkrylov_hip.so; else LIB=$PWD/build/$v/libkrylov_hip.so; fi
  KT_LIB=$LIB timeout -k 10 120 python tools/ky_diag.py $v >> $O/timing.jsonl 2> $O/$v.err
  tail -1 $O/timing.jsonl
  i=0
  for pmc in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    KT_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-include-regex "k_spmm_lanczos<" -d $O/${v}_p$i -o c --output-format csv -- python3 tools/ky_diag.py $v > $O/${v}_p$i.log 2>&1
    python3 tools/ky_diag_pmc.py $O/pmc.json $v $(find $O/${v}_p$i -name "*counter_collection.csv")
  done
done
