"""Mirror of the reference's ``modules`` package (src/modules/): same class names, constructor
arguments, attributes and state_dict keys; the step runs on the MI355X HIP kernels."""
from .graph_augmentation import GraphAugmentation
from .nca import NeuralCA
from .ncagraph import NeuralCAGraph
from .perception import FixedSobelPerception

__all__ = ["FixedSobelPerception", "NeuralCA", "GraphAugmentation", "NeuralCAGraph"]
