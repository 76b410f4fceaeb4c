"""MI355X-native NCA rollout step (Psylocibe23/Graph_Neural_Cellular_Automata hot path).

The HIP kernels live in csrc/ and are built into libgnca.so (C ABI: include/gnca.h).  The
``modules`` subpackage mirrors the reference's nn.Module API on top of it.
"""
from .modules import FixedSobelPerception, GraphAugmentation, NeuralCA, NeuralCAGraph

__all__ = ["FixedSobelPerception", "NeuralCA", "GraphAugmentation", "NeuralCAGraph"]
