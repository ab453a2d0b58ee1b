"""``com.linkedin.tony.cli.LocalSubmitter``: local (CPU, fake GPU inventory) mode."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))))))

from tony_amd.cli.local_submitter import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main() & 0xFF)
