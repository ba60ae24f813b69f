"""Drop-in import name: ``import dbscan`` / ``from dbscan import DBSCAN``
resolve to the MI355X implementation (pypardis_amd), mirroring
R:dbscan/__init__.py.  Submodule paths (``dbscan.partition``, ...) alias too."""
import sys as _sys

import pypardis_amd as _impl
from pypardis_amd import *  # noqa: F401,F403
from pypardis_amd import (__version__, ClusterAggregator, default_value, BoundingBox,  # noqa: F401
                          median_search_split, mean_var_split, min_var_split, KDPartitioner,
                          dbscan_partition, map_cluster_id, DBSCAN)
from pypardis_amd import aggregator, geometry, partition  # noqa: F401
from pypardis_amd import dbscan as _dbscan_mod

for _name, _mod in (("aggregator", aggregator), ("geometry", geometry),
                    ("partition", partition), ("dbscan", _dbscan_mod)):
    _sys.modules[__name__ + "." + _name] = _mod
