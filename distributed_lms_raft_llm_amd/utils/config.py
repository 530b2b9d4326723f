"""Config files for the server CLIs (the reference hard-codes every address and
constant, §2.7).  A YAML or JSON file supplies defaults for any command-line flag (``data-dir`` or
``data_dir``); explicit flags still win.  The LMS server additionally understands a cluster map:

    servers: {1: "10.0.0.1:50051", 2: "10.0.0.2:50052", 3: "10.0.0.3:50053"}
    tutor: "10.0.0.9:50054,10.0.0.10:50054"     # tutoring replicas (failover order)
    gate: bert
    gate_threshold: 0.6
    election_timeout: "0.15,0.30"

so every node starts with ``lms_server.py --config cluster.yaml <id>`` and derives its port and
its peers (keyed by their real ids) from the same file.
"""
from __future__ import annotations

import argparse
import json
import os


def load_config(path: str) -> dict:
    with open(path) as f:
        text = f.read()
    if path.endswith((".yaml", ".yml")):
        import yaml

        data = yaml.safe_load(text) or {}
    else:
        data = json.loads(text)
    if not isinstance(data, dict):
        raise ValueError(f"{path}: top level must be a mapping")
    return data


def parse_with_config(parser: argparse.ArgumentParser, argv=None) -> tuple[argparse.Namespace, dict]:
    """Parse ``argv`` with defaults taken from ``--config FILE`` (or ``$DLMS_CONFIG``)."""
    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("--config", default=os.environ.get("DLMS_CONFIG"))
    known, _ = pre.parse_known_args(argv)
    parser.add_argument("--config", default=known.config, help="YAML/JSON file with flag defaults")
    cfg = load_config(known.config) if known.config else {}
    dests = {a.dest for a in parser._actions}
    defaults = {}
    for k, v in cfg.items():
        d = str(k).replace("-", "_")
        if d in dests:
            defaults[d] = v
    parser.set_defaults(**defaults)
    return parser.parse_args(argv), cfg
