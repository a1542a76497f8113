"""TFPark text models (Py/tfpark/text/**): BERT estimators and Keras text models,
built on this framework's BERT / LSTM / CRF ops instead of TensorFlow."""
