from zoo.tfpark.text.keras.intent_extraction import IntentEntity  # noqa: F401
from zoo.tfpark.text.keras.ner import NER  # noqa: F401
from zoo.tfpark.text.keras.pos_tagging import POSTagger, SequenceTagger  # noqa: F401
from zoo.tfpark.text.keras.text_model import CRF, TextKerasModel  # noqa: F401
