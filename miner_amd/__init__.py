"""miner_amd — MINER's multi-interest scoring path, MI355X-native.

PolyAttention -> TargetAwareAttention -> candidate ranking as one fused HIP kernel for gfx950
(``csrc/miner_score.hip``, C ABI in ``include/miner_score.h``), behind a drop-in mirror of the
reference's ``src/model/model.py`` modules and ``src/evaluation.py`` evaluator.

Modules:
  model       Miner / PolyAttention / TargetAwareAttention (reference nn.Module contract + score())
  ops         torch-facing wrappers of the C ABI
  evaluation  SlowEvaluator / FastEvaluator and metric functions (reference evaluator contract)
  synthetic   counter-keyed synthetic MIND-shaped impressions
  distributed impression sharding + RCCL reduction of metric partials
  main        `main.py eval`-compatible driver (python -m miner_amd.main eval ...)
"""
__version__ = "0.1.0"
