"""ORACLE — test infrastructure only.

CPU restatement of the reference's hot path, used ONLY by ``tests/``,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` as
the checker / CPU baseline.  Nothing in the product package imports it; the
product path has no CPU fallback.

Pinning: ``tests/test_oracle.py`` checks these functions against the golden
vectors in ``tests/golden/`` that ``tests/golden/make_golden.py`` recorded by
running the reference itself in the build container (R8 graph rebuilt by the
reference's builder; logits of the reference GCN for three seeds, a
train-mode forward/backward, two full training runs, tiny known-answer
graphs).  The reference ships no tests or fixtures of its own for this path
(SURVEY.md §4), so those generated goldens are the pin.

Modules:
  gcn_ref   torch-CPU restatement issuing the same ATen calls as layer.py
            (th.spmm on the COO tensors as utils.py/trainer.py lay them out)
            plus the trainer loop (trainer.py:349-406) and metrics.
  csr_ref   numpy float64 restatement from the math (CSR SpMM, adjacency
            normalisation, GEMM, column sums) for kernel-level parity.
  spmm_ref.c  plain-C CSR SpMM (double accumulation) for large parity cases,
            built into oracle/liboracle.so by __graft_entry__.build().
"""
