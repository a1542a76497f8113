from zoo.tfpark.text.estimator.bert_base import (BERTBaseEstimator, BertConfig, BertEncoder,  # noqa: F401
                                                 bert_input_fn, build_bert, load_bert_checkpoint)
from zoo.tfpark.text.estimator.bert_classifier import BERTClassifier  # noqa: F401
from zoo.tfpark.text.estimator.bert_ner import BERTNER  # noqa: F401
from zoo.tfpark.text.estimator.bert_squad import BERTSQuAD  # noqa: F401
