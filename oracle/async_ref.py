"""numpy arithmetic of the reference's asyncio agent step (TEST INFRASTRUCTURE ONLY).

The same interface as ``distributed_learning_amd.iterates.DeviceIterates``, with the
reference's own numpy expressions, so that tests can drive the façade's message protocol
(utils/consensus_asyncio.py) on the CPU and compare the schedule with the reference-generated
fixtures without a GPU.  Never used by the product path (it does not import this package).

  load    y = value * weight / mean_weight                    consensus_asyncio.py:231
  update  y * (1 - eps*deg) + eps * np.sum(values, axis=0)    :295
          np.all([(y - v) <= convergence_eps for v in values]) :297
"""
import numpy as np


class NumpyIterates:
    def __init__(self):
        self.updates = 0

    def load(self, value, weight, mean_weight):
        return value * weight / mean_weight

    def update(self, y, nbrs, keep, eps, conv_eps):
        y = y * keep + eps * np.sum(nbrs, axis=0)
        self.updates += 1
        return y, bool(np.all([(y - v) <= conv_eps for v in nbrs]))

    def result(self, y):
        return y
