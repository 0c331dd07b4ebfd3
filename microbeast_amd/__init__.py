"""microbeast_amd — MI355X-native IMPALA actor-learner for (synthetic) gym-microRTS.

A from-scratch re-design of Neos-codes/microbeast for AMD Instinct MI355X
(gfx950): native C++ env + actor engine, hand-written HIP kernels for the hot
ops, RCCL data-parallel learners. See README.md and SURVEY.md.
"""
__version__ = "0.1.0"
