"""``com.linkedin.tony.cli.NotebookSubmitter``: single-node notebook job + local port forward."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))))))

from tony_amd.cli.notebook_submitter import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main() & 0xFF)
