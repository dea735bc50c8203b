"""Reference-compatible module path (reference dataset.py)."""
from pyrecover_amd.data.dataset import CollatorForCLM, ParquetDataset, SyntheticTokenDataset  # noqa: F401
