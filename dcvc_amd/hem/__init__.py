"""DCVC-HEM on MI355X: DMC (P-frame) and IntraNoAR (I-frame) with the
reference's API (DCVC-HEM/src/models/video_model.py, image_model.py)."""
from .video_model import DMC  # noqa: F401
from .image_model import IntraNoAR  # noqa: F401
