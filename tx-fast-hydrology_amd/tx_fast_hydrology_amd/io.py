"""JSON encoding of model descriptions (reference ``tx_fast_hydrology/io.py:1-47``).

``ModelEncoder`` turns timestamps and timedeltas into ISO-8601 strings and arrays into lists;
``ModelDecoder`` turns the typed fields of a model description back into numpy arrays
(``startnodes``/``endnodes`` int64, ``K``/``X``/``o_t`` float64) and pandas time objects, at any
nesting depth (collections nest model descriptions under ``models/<name>/model``).
"""
import json

import numpy as np
import pandas as pd

DEFAULT_START_TIME = pd.to_datetime(0.0, utc=True)
DEFAULT_TIMEDELTA = pd.to_timedelta(3600, unit="s")

_INT_FIELDS = ("startnodes", "endnodes")
_FLOAT_FIELDS = ("K", "X", "o_t")


def _decode_field(key, value):
    if key in _INT_FIELDS:
        return np.asarray(value, dtype=np.int64)
    if key in _FLOAT_FIELDS:
        return np.asarray(value, dtype=np.float64)
    if key == "datetime":
        return pd.to_datetime(value)
    if key == "timedelta":
        return pd.to_timedelta(value)
    return value


class ModelEncoder(json.JSONEncoder):
    """JSON encoder for model descriptions (``Muskingum.info``)."""

    def default(self, obj):
        if isinstance(obj, (pd.Timestamp, pd.Timedelta)):
            return obj.isoformat()
        if isinstance(obj, np.ndarray):
            return obj.tolist()
        return super().default(obj)


class ModelDecoder(json.JSONDecoder):
    """JSON decoder restoring the typed fields of model descriptions."""

    def __init__(self, *args, **kwargs):
        kwargs["object_hook"] = self._typed
        super().__init__(*args, **kwargs)

    @staticmethod
    def _typed(obj):
        return {key: _decode_field(key, value) for key, value in obj.items()}
