from .mixer import *  # noqa: F401,F403  (mirrors reference utils/consensus_simple/__init__.py)
