"""TextClassifier (Zs/models/textclassification/TextClassifier.scala:34-192,
Py text_classifier.py:29-170): WordEmbedding -> CNN / LSTM / GRU encoder ->
Dense(128) -> Dropout(0.2) -> ReLU -> Dense(class_num, softmax)."""
from zoo.models.common.zoo_model import ZooModel
from zoo.pipeline.api.keras.layers import (GRU, LSTM, Activation, Convolution1D, Dense, Dropout, Embedding,
                                           GlobalMaxPooling1D, WordEmbedding)
from zoo.pipeline.api.keras.models import Sequential


class TextClassifier(ZooModel):
    def __init__(self, class_num, embedding_file=None, word_index=None, sequence_length=500, encoder="cnn",
                 encoder_output_dim=256, vocab_size=None, embed_dim=None, **kwargs):
        super().__init__(**kwargs)
        self.class_num, self.sequence_length = int(class_num), int(sequence_length)
        self.encoder, self.encoder_output_dim = encoder.lower(), int(encoder_output_dim)
        if embedding_file is not None:
            self.embedding = WordEmbedding(embedding_file, word_index, input_length=sequence_length)
        elif vocab_size is not None and embed_dim is not None:
            self.embedding = Embedding(int(vocab_size), int(embed_dim), input_length=sequence_length)
        else:
            raise ValueError("TextClassifier needs embedding_file (GloVe text) or vocab_size + embed_dim")
        if self.encoder not in ("cnn", "lstm", "gru"):
            raise ValueError("Unsupported encoder for TextClassifier: " + encoder)
        self._init_model()

    def build_model(self):
        m = Sequential()
        m.add(self.embedding)
        if self.encoder == "cnn":
            m.add(Convolution1D(self.encoder_output_dim, 5, activation="relu"))
            m.add(GlobalMaxPooling1D())
        elif self.encoder == "lstm":
            m.add(LSTM(self.encoder_output_dim))
        else:
            m.add(GRU(self.encoder_output_dim))
        m.add(Dense(128))
        m.add(Dropout(0.2))
        m.add(Activation("relu"))
        m.add(Dense(self.class_num, activation="softmax"))
        return m
