"""dcvc_amd — MI355X-native (gfx950) engine for the DCVC-DC / DCVC-HEM
contextual encode/decode hot path.  See DESIGN.md."""
__version__ = "0.1.0"
