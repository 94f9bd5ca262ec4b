"""research_image_retrieval_amd — MI355X-native embed+search hot path of
Mak-GIBA/research_image_retrieval (src/benchmark), behind the reference's own
extractor / ranker API.  Kernels: librr.so (hand-written HIP for gfx950)."""
__version__ = "0.1.0"
