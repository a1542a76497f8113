"""Runnable examples (the reference's pyzoo/zoo/examples and Zs/examples): every script
has a ``main(argv)`` that runs end to end on synthetic data (there is no network here for
datasets), on the GPU when one is present and on the CPU otherwise.

    python analytics-zoo_amd/examples/resnet/train_imagenet.py --help
"""
