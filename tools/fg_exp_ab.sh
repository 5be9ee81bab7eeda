# fun_and_grad_krylov_exp on India (the Hessian driver's setting): which round-3 change moved it?
set -e
O=gpurun_out/fgexp; mkdir -p $O
run() { local tag=$1; shift; env "$@" timeout -k 10 120 python tools/prof_fg_exp.py > $O/$tag.txt 2>&1; echo "== $tag"; grep fg_exp $O/$tag.txt; }
run base KT_DUMMY=1
run nopipe KT_FU_PIPE=0 KT_TFU_PIPE=0
run nochol KT_QR_CHOL=0
run nopow KT_NORM_POW=0
run rocblas KT_GEMM_ROCBLAS=1
run all_old KT_FU_PIPE=0 KT_TFU_PIPE=0 KT_QR_CHOL=0 KT_NORM_POW=0 KT_GEMM_ROCBLAS=1
run timing KT_FG_TIMING=1
KT_DUMMY=1 timeout -k 10 120 python tools/prof_fg_exp.py --hess > $O/hess.txt 2>&1; grep hessian $O/hess.txt
