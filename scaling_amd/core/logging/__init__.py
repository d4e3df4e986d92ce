from .logger_config import LoggerConfig, LogLevel
from .logging import ColorFormatter, Logger, logger

__all__ = ["ColorFormatter", "Logger", "LoggerConfig", "LogLevel", "logger"]
