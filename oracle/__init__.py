"""CPU oracle for the art-sbir hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this package, and only as the checker / the timed CPU baseline.
The product path (``art-sbir_amd/``) never imports, links or calls it.

Contents
  encoder.py   — CPU fp32 restatement of models.py:191-379 (ModifiedResNet,
                 Bottleneck, AttentionPool2d, the classification head) on plain
                 torch ops, same constructor signatures and state_dict keys.
  steps.py     — the triplet training step of train.py:27-37,59-70 with
                 nn.TripletMarginLoss / optim.Adam, deterministic init.
  retrieval.py — inference.py:30-69,94-136 + utils.py:22-25 (rank of the
                 positive, top-k, MRR, top-k accuracy, describe() stats) in
                 numpy float64.
  numpy_ref.py — an independent float64 numpy restatement of the forward ops
                 (conv, batch-norm, attention pool, triplet loss, Adam) used
                 to cross-pin encoder.py/steps.py.

Parity status: the reference publishes no tests, fixtures or golden vectors,
and importing/running the reference in this container was refused by the
environment.  The oracle is therefore "parity unpinned" with
respect to the reference itself; it is cross-pinned between two independent
restatements (torch.nn ops vs numpy float64) — see tests/test_oracle.py.
The arithmetic lives in PyTorch (third-party; reference unpinned, restated
against torch 2.10.0 defaults: PairwiseDistance eps=1e-6 on (x1-x2+eps),
BatchNorm eps=1e-5 momentum=0.1, Adam betas=(0.9,0.999) eps=1e-8 coupled L2).
"""
