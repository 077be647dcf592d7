from .base_config import BaseConfig
from .my_config import MyConfig
from .optuna_config import OptunaConfig
from .parser import get_parser, load_parser

__all__ = ['BaseConfig', 'MyConfig', 'OptunaConfig', 'get_parser', 'load_parser']
