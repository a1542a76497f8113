"""Py/util/tf.py: ``export_tf`` freezes a live TF session into the folder layout
TFNet loads (frozen_inference_graph.pb + graph_meta.json). It needs TensorFlow
itself; graphs exported elsewhere load with zoo.tfpark.TFNet."""


def export_tf(sess, folder, inputs, outputs, generate_backward=False, allow_non_differentiable_input=True):
    raise NotImplementedError("export_tf needs a TensorFlow session; load exported folders / SavedModels "
                              "with zoo.tfpark.TFNet")
