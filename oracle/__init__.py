"""CPU oracle for the trace(f(A)) path -- test infrastructure only.

Importable by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
only.  krylov_oracle.py restates the reference's MATLAB algorithms in NumPy;
slq_ref.c restates the probe-Lanczos path in C (OpenMP) for the CPU baseline.
Parity is pinned to the reference's known-answer identities (exact dense
traces) since the MATLAB reference cannot run here and ships no golden
vectors (see krylov_oracle.py header).
"""
