from .paths import BIN_DIR, BUILD_DIR, LIB_DIR, bin_path, is_built, lib_path
from .log import log, verbose

__all__ = ["BIN_DIR", "BUILD_DIR", "LIB_DIR", "bin_path", "is_built", "lib_path", "log", "verbose"]
