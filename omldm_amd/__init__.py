"""omldm_amd — MI355X-native streaming online machine learning engine with the
capabilities of ArisKonidaris/OMLDM (see README.md)."""
__version__ = "0.1.0"
