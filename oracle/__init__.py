"""TEST INFRASTRUCTURE ONLY — the CPU oracle for the Siamese GCN→NTN hot path.

Nothing in ``graphembedding_amd`` (the product) may import, link or execute
anything under ``oracle/``.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` use it, and only as the checker / the timed
CPU baseline.

Contents
  siamese_oracle.py  float64 numpy restatement of the TensorFlow math of
                     /root/reference/model/Siamese (layers.py, models.py,
                     model_mse.py), every quirk of SURVEY.md Appendix A included,
                     plus the counter-based dropout RNG the HIP kernels share.
  siamese_cpu.c      the same math in C (float32, OpenMP over pairs) — the timed
                     CPU baseline ("kind": "port") of bench.py.

Pinning status
  * graph preprocessing, one-hot encoding, the RandomSampler/DistributionSampler
    pair streams, GaussianKernel and normalized_dist are pinned bit-exactly by
    fixtures generated from the reference's own modules in this container
    (tests/golden/make_golden.py).
  * The TF layer math itself is "parity unpinned" by the reference: TensorFlow is
    not installed here (ModuleNotFoundError, not a permission denial) and the
    reference holds no golden vectors.  The restatement is cross-validated by an
    independent torch-autograd implementation and by finite differences.
"""
