"""Print the Scv CustomResourceDefinition (deploy/scv-crd.yaml is generated from this)."""
import sys

import yaml

from .scv import crd_manifest

if __name__ == "__main__":
    yaml.safe_dump(crd_manifest(), sys.stdout, sort_keys=False)
