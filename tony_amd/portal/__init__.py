"""History portal + history maintenance (tony-portal)."""
from .history import HistoryFileMover, HistoryFilePurger, purge_finished_dir, purge_intermediate_dir
from .server import CacheWrapper, PortalServer

__all__ = ["HistoryFileMover", "HistoryFilePurger", "purge_finished_dir", "purge_intermediate_dir",
           "CacheWrapper", "PortalServer"]
