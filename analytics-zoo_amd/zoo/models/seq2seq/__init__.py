from zoo.models.seq2seq.seq2seq import Bridge, RNNDecoder, RNNEncoder, Seq2seq  # noqa: F401
