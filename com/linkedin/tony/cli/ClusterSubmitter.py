"""``com.linkedin.tony.cli.ClusterSubmitter``: TonY's CLI entry point, served by tony_amd."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))))))

from tony_amd.cli.cluster_submitter import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main() & 0xFF)
