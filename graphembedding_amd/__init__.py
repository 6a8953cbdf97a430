"""graphembedding_amd — MI355X-native Siamese graph-similarity training engine.

Drop-in for the hot path of kangzf/GraphEmbedding's model/Siamese (GCN →
pooling → NTN → Gaussian similarity → MSE, forward + backward + Adam): host
code in Python mirrors the reference's interfaces (config/layer grammar,
graphs, samplers, data, similarity, distance, results, metrics), and the
arithmetic runs in libsiamese_hip.so (hand-written gfx950 HIP kernels behind
the C-ABI of include/siamese_hip.h).
"""
__version__ = '0.1.0'
