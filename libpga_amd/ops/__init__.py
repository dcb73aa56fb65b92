"""Device operators and genome codecs."""
from .codec import decode, encode  # noqa: F401
