# Cross-process A/B of two library builds (KT_LIB) on config 3's fun_and_grad_krylov_fun, alternating 3x.
set -o pipefail
for r in 1 2 3; do
  for L in ablib/libkrylov_prev.so krylov_robustness_amd/libkrylov_hip.so; do
    echo "$L $(KT_LIB=$PWD/$L timeout -k 10 120 python tools/fg_ab_inproc.py 24 KT_AB_DUMMY=0 2>/dev/null | grep median)"
  done
done
