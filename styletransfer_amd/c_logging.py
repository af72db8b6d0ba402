"""Logging (mirror of stransfer/c_logging.py): the 'StyleTransfer' logger with a
tqdm-safe stream handler and a `runs/runtime.log` file handler."""
import logging
import os

import tqdm

from . import constants

_LOGGER = logging.getLogger("StyleTransfer")
_LOGGER.setLevel(logging.INFO)
_LOGGER.handlers = []

LOGGER_FORMATTER = logging.Formatter(
    "%(asctime)s [%(levelname)s] %(module)s.%(funcName)s #%(lineno)d - %(message)s")


class TqdmLoggingHandler(logging.StreamHandler):
    """Writes through tqdm so progress bars stay at the bottom."""

    def emit(self, record):
        try:
            tqdm.tqdm.write(self.format(record))
            self.flush()
        except (KeyboardInterrupt, SystemExit):
            raise
        except Exception:
            self.handleError(record)


tqdm_handler = TqdmLoggingHandler()
tqdm_handler.setFormatter(LOGGER_FORMATTER)
_LOGGER.addHandler(tqdm_handler)

if os.environ.get("STX_NO_LOGFILE") != "1":
    try:
        os.makedirs(constants.RUNS_PATH, exist_ok=True)
        file_handler = logging.FileHandler(constants.LOG_PATH, mode="w+")
        file_handler.setFormatter(LOGGER_FORMATTER)
        _LOGGER.addHandler(file_handler)
    except OSError:  # read-only working directory: stream logging only
        pass


def get_logger() -> logging.Logger:
    return _LOGGER
