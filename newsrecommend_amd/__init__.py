"""newsrecommend_amd — MI355X-native hot path of YuxuanZhao/NewsRecommend.

  newsrecommend_amd.faiss  : faiss-compatible exact flat indexes (IndexFlatIP /
                             IndexFlatL2) on bf16-MFMA screening + fp64 rescoring
  newsrecommend_amd.din    : DIN ranker (AttentionLayer, DIN, train, evaluate)
                             with the attention pool in HIP kernels
  newsrecommend_amd.data   : dataset restatements + synthetic workloads
  newsrecommend_amd.dist   : corpus sharding over ranks + RCCL top-k merge

Kernels live in libnrk.so (include/nrk.h), built by newsrecommend_amd.build.
"""
__version__ = "0.1.0"
