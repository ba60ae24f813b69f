"""pypardis_amd — MI355X-native drop-in for the pyParDis DBSCAN hot path.

Same export surface as the reference package (R:dbscan/__init__.py:1-21).
All clustering runs as HIP kernels in libpardis.so (see include/pardis.h);
there is no CPU fallback.
"""
__version__ = (0, 1, 0)

from .aggregator import (
    ClusterAggregator,
    default_value
)
from .geometry import (
    BoundingBox
)
from .partition import (
    median_search_split,
    mean_var_split,
    min_var_split,
    KDPartitioner
)
from .dbscan import (
    dbscan_partition,
    map_cluster_id,
    DBSCAN
)
