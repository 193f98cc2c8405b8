"""H2O-compatible Python API backed by the MI355X-native engine (``llama_github_io_amd``)."""
__version__ = "3.46.0.amd0"
