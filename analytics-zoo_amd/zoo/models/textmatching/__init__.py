from zoo.models.textmatching.knrm import KNRM, KernelPooling  # noqa: F401
from zoo.models.textmatching.text_matcher import TextMatcher, prepare_embedding  # noqa: F401
