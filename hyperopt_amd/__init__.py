"""hyperopt_amd -- MI355X-native TPE suggestion engine with hyperopt's API."""
__version__ = '0.1.0'
