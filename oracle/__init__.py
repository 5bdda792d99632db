"""CPU oracle for the HD-GNN training step -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may import anything from this package, and only as the checker
(or, for ``cpu_baseline``, as the CPU path being timed).  The product path
(``hd-gnn_amd/hdgnn``) never imports it and fails loudly when its HIP
extension is missing.

Contents
--------
``layout``     variable order / shapes of model_1..4 (tf.global_variables order).
``model_ref``  pair-explicit torch-CPU restatement of model_{1,2,3,4}.build_model
               (forward + the three loss terms); gradients come from
               torch.autograd, Adam is restated from TF1's ApplyAdam.
``literal``    literal incidence-matrix restatement (Es/Et/Cs/Ct/Esc/Etc dense
               batched matmuls, op for op as model_2.py writes them).  Same
               FLOPs as the TF graph; used as the CPU baseline ("port").
``loader_ref`` restatement of utils2.read_data's bookkeeping in compact form
               (x, a, y, hunk-id maps), pinned bit-exact against golden
               vectors produced by running the reference utils2.py itself.

Parity status
-------------
* Loader bookkeeping: PINNED (tests/golden/loader_tiny.npz, produced by the
  reference utils2.read_data on a synthetic tree; tools/gen_loader_golden.py).
* Model arithmetic: PARITY UNPINNED against TensorFlow.  TensorFlow is not
  installed in this image (``import model_2`` raises ModuleNotFoundError) and the
  reference ships no tests or golden outputs, so the TF op semantics are restated
  from model_2.py (file:line cited at every stage) and cross-checked between two
  independent restatements (``literal`` vs ``model_ref``).
"""
