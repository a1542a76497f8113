from zoo.feature.text.text_set import (DistributedTextSet, LocalTextSet, Normalizer, Relation,  # noqa: F401
                                       SequenceShaper, TextFeature, TextFeatureToSample, TextSet, Tokenizer,
                                       WordIndexer, generate_relation_pairs)
