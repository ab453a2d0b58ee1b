"""TonY-compatible module path (see tony_amd.cli)."""
