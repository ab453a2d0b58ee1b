"""Configuration system: Hadoop-XML loader + the tony.* key schema."""
from . import keys  # noqa: F401
from .configuration import DEFAULT_XML, Configuration, ConfigurationError  # noqa: F401
