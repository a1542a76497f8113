"""Every example under analytics-zoo_amd/examples runs end to end (tiny arguments, CPU)."""
import importlib.util
import os

import pytest

EX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "analytics-zoo_amd", "examples")

CASES = [
    ("resnet/train_imagenet.py", ["--depth", "18", "--classes", "10", "--image-size", "32", "--batch", "4",
                                  "--iters", "2", "--width", "8"]),
    ("lenet/lenet_keras.py", ["--n", "256", "--epochs", "1"]),
    ("recommendation/ncf.py", ["--users", "200", "--items", "100", "--n", "2000", "--batch", "256", "--epochs", "1"]),
    ("recommendation/wide_n_deep.py", ["--n", "300", "--epochs", "1"]),
    ("textclassification/text_classification.py", ["--n", "100", "--epochs", "1", "--sequence-length", "16"]),
    ("anomalydetection/anomaly_detection.py", ["--n", "300", "--epochs", "1"]),
    ("autograd/custom_loss.py", ["--n", "200", "--epochs", "2"]),
    ("nnframes/image_transfer_learning.py", ["--epochs", "2"]),
    ("tfpark/keras_ndarray.py", ["--n", "128", "--epochs", "1", "--use-dataset"]),
    ("pytorch/simple_training.py", ["--n", "128", "--epochs", "2"]),
    ("xshard/pandas_xshards.py", ["--files", "3"]),
    ("ray/parameter_server.py", ["--iters", "3"]),
    ("qaranker/qa_ranker.py", ["--questions", "8", "--epochs", "1"]),
    ("serving/quick_start.py", ["--images", "4", "--batch", "2"]),
    ("attention/transformer.py", ["--n", "32", "--epochs", "1", "--seq-len", "8", "--hidden", "16"]),
    ("objectdetection/ssd_train_predict.py", ["--steps", "1", "--batch", "1"]),
    ("imageclassification/predict.py", ["--images", "2", "--model", "squeezenet"]),
    ("inception/inception.py", ["--batch", "2", "--iters", "2", "--classes", "10", "--image-size", "64"]),
    ("quantization/quantized_inference.py", ["--depth", "18", "--batch", "2", "--image-size", "64"]),
    ("streaming/streaming_text_classification.py", ["--lines", "12", "--micro-batch", "4", "--epochs", "2"]),
    ("openvino/predict.py", ["--batch", "2"]),
]


@pytest.mark.parametrize("path,args", CASES, ids=[c[0] for c in CASES])
def test_example_runs(path, args):
    spec = importlib.util.spec_from_file_location("ex_" + path.replace("/", "_")[:-3], os.path.join(EX, path))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert mod.main(args) is not None
