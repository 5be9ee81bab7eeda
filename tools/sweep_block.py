"""Time kt_slq_trace per probe-block width P on a config graph (GPU box)."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="sf1m")
    ap.add_argument("--nprobes", type=int, default=256)
    ap.add_argument("--m", type=int, default=30)
    ap.add_argument("--blocks", default="4,8,16,32,64,128")
    ap.add_argument("--variants", default="relabel", help="comma list: relabel,natural")
    a = ap.parse_args()
    import krylov_robustness_amd as kra
    from krylov_robustness_amd import graphs
    t = time.time()
    if a.config == "sf1m":
        A = graphs.chung_lu(1_000_000, 10_000_000, seed=0)
    else:
        A = graphs.erdos_renyi(100_000, 500_000, seed=0)
    print(f"graph {a.config} n={A.shape[0]} nnz={A.nnz} gen {time.time()-t:.1f}s", flush=True)
    n, nnz = A.shape[0], A.nnz
    for var in a.variants.split(","):
      os.environ["KT_RELABEL"] = "0" if var == "natural" else "1"
      os.environ["KT_K1_FLAGS"] = {"nt": "1", "mlp": "4", "mlpnt": "5", "nty": "8", "ntboth": "9",
                                   "ntall": "9", "ntyk2": "8", "mlpk2": "12"}.get(var.split("_")[0], "0")
      os.environ["KT_K2_NT"] = "1" if var.startswith(("k2nt", "ntall", "ntyk2", "mlpk2")) else "0"
      os.environ["KT_SLQ_LANES"] = (var[5:] if var.startswith("lanes")
                                    else var.split("_lanes")[1] if "_lanes" in var else "1")
      os.environ["KT_UNIT"] = "0" if var == "valued" else "1"
      # y-form variants: "y", "ynt" (nontemporal y_{j+1} store), "ysc1" (write-through
      # y_{j+1} store), "_lanesL" suffix
      os.environ["KT_SLQ_YFORM"] = "1" if var.startswith("y") else "0"
      os.environ["KT_KY_FLAGS"] = ("8" if var.startswith("ynt") else "16" if var.startswith("ysc1")
                                   else "0")
      if var.startswith("y"):
          os.environ["KT_K1_FLAGS"] = "8"
          os.environ["KT_K2_NT"] = "1"
      ctx = kra.Context(0)
      D = kra.DeviceMatrix(A, ctx)
      print(f"--- variant {var}", flush=True)
      for P in [int(x) for x in a.blocks.split(",")]:
          kra.slq_quadforms(D, P, 4, seed=0, block=P, ctx=ctx)  # warm
          ctx.profile_reset(); ctx.profile(True)
          t = time.perf_counter()
          s1, _, q = kra.slq_quadforms(D, a.nprobes, a.m, seed=0, block=P, ctx=ctx)
          el = time.perf_counter() - t
          ctx.profile(False)
          l1, ms1 = ctx.profile_read(0)
          l2, ms2 = ctx.profile_read(1)
          k1 = ms1 / max(l1, 1); k2 = ms2 / max(l2, 1)
          k1_bytes = 12 * nnz + 4 * (n + 1) + 16 * n * P
          k2_bytes = 32 * n * P
          per_eval_1024 = el / a.nprobes * 1024
          print(f"P={P:4d} total {el*1e3:9.1f} ms  ({1/per_eval_1024:7.3f} evals/s @1024 probes) "
                f"K1 {k1*1e3:8.1f} us {k1_bytes/k1/1e6:7.0f} GB/s  K2 {k2*1e3:8.1f} us "
                f"{k2_bytes/max(k2, 1e-9)/1e6:7.0f} GB/s  launches {l1}  K1+K2 share {(ms1+ms2)/(el*1e3):.2f}  "
                f"tr~{s1/a.nprobes:.4e}  redone {ctx.yform_redone()}", flush=True)


if __name__ == "__main__":
    main()
