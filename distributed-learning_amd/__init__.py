"""MI355X-native consensus (gossip) learning engine.

Drop-in for the data-parallel hot path of Malkovsky/distributed-learning: many simulated agents
hold flattened parameter vectors and alternate a local gradient step with a gossip mix
``X <- W X`` over a sparse graph.  The hot path runs in hand-written HIP kernels for gfx950
(``csrc/``, built into ``_lib/libdlamd.so``) behind a C ABI (``include/dlamd.h``); this package
is the host layer that mirrors the reference's Python API:

* ``utils.consensus_simple.Mixer``            (reference utils/consensus_simple/mixer.py)
* ``utils.consensus_asyncio``                  (reference utils/consensus_asyncio.py)
* ``utils.fast_averaging.find_optimal_weights`` (reference utils/fast_averaging.py)
* ``networks.ANNModel`` / ``networks.LogRegTitanic`` (reference networks/)
* ``engine.GossipEngine``: device-resident agent matrix + fused round (the bench/trainer core)
* ``sharding``: multi-GPU column-stripe and agent-partition (halo exchange) execution
"""
__version__ = "0.1.0"
