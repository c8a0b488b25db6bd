"""gpboost_amd — MI355X-native GP likelihood engine behind GPBoost's C API.

The compute path is the in-tree HIP library gpboost_amd/lib/libgpboost_amd.so
(build: ``python -m gpboost_amd.build``); this package is the host-side mirror of the
reference Python ``GPModel`` for the likelihood path.
"""
from .basic import GPBoostError, GPModel, combine_partials, comm_create_id, partition_rows  # noqa: F401

__all__ = ["GPModel", "GPBoostError", "combine_partials", "comm_create_id", "partition_rows"]
