"""Per-class loggers (reference ``utils.py:281-302``)."""
from __future__ import annotations

import logging
import os
import sys
from typing import Union


def get_logger(cls: Union[type, str], level: str = "INFO") -> logging.Logger:
    name = cls if isinstance(cls, str) else cls.__name__
    logger = logging.getLogger("srml." + name)
    if not logger.handlers:
        handler = logging.StreamHandler(sys.stderr)
        handler.setFormatter(logging.Formatter("%(asctime)s - %(name)s - %(levelname)s - %(message)s"))
        logger.addHandler(handler)
        logger.propagate = False
    logger.setLevel(os.environ.get("SRML_LOG_LEVEL", "WARNING"))
    return logger
