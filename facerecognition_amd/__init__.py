"""facerecognition_amd — MI355X-native face-embedding extraction + gallery match.

Drop-in for the hot path of sin0235/FaceRecognition (inference/extract_embeddings.py +
inference/recognition_engine.py + inference/database_builder.py): the Python API keeps the
reference's names and behaviour, the compute runs in the C-ABI HIP library libfrhip.so
(include/frhip.h).  See DESIGN.md.
"""
from .weights import ARCHS, INPUT_SIZE  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):  # lazy: importing the package must not initialise the GPU
    if name == "FRModel":
        from .model import FRModel
        return FRModel
    if name == "DeviceGallery":
        from .gallery import DeviceGallery
        return DeviceGallery
    raise AttributeError(name)
