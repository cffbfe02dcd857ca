"""CPU oracle for the scgpu hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
anything under oracle/. The product package (gym-supplychain_amd/) never imports it
and has no CPU fallback: it fails loudly when its HIP library is missing.

Contents
  philox.py        Philox4x32-10 restatement (numpy), pinned by Random123 known-answer vectors
  poisson.py       Poisson(lambda) uint32 inverse-CDF threshold table + inversion
  beergame.py      per-env NumPy restatement of BeerGameEnv (beergame_env.py:11-181),
                   pinned against golden vectors generated from the reference itself
  beergame_oracle.c  batched C restatement of the same step (fast checker for large N)
  gen_golden.py    imports /root/reference (this container only) and writes tests/golden/
"""
