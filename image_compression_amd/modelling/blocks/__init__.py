from .entropy_model import EntropyModel, GaussianConditionalModel, LaplacianConditionalModel
from .prior_analysis import HyperpriorAnalysisTransform
from .prior_synthesis import HyperpriorSynthesisTransform
from .analysis import AnalysisTransform
from .synthesis import SynthesisTransform
from .build import ENTROPY_MODEL_REGISTRY
