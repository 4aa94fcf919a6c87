"""Host-side mirror of OpenTSDB's aggregation interface (names, argument
meaning and error behaviour of the reference), backed by the HIP engine.

Mirrors:
  Aggregators / Aggregator / Interpolation   src/core/Aggregators.java:33-228
  FillPolicy                                 src/core/FillPolicy.java:22-62
  DateTime.parseDuration                     src/utils/DateTime.java:187-231
  DownsamplingSpecification                  src/core/DownsamplingSpecification.java:116-191
  RateOptions                                src/core/RateOptions.java:27-176
  TsdbQuery scan bounds                      src/core/TsdbQuery.java:1573-1675
  AggregationIterator.create / SpanGroup     src/core/AggregationIterator.java:351-380,
                                             src/core/SpanGroup.java:253-339,525-530
Only spec parsing and array plumbing live here; every data point is computed
by libotsdb_agg.so on the GPU (opentsdb_amd.engine).
"""
from enum import IntEnum

LONG_MAX = 2**63 - 1
SECOND_MASK = 0xFFFFFFFF00000000
MAX_TIMESPAN = 3600


# --------------------------------------------------------------- exceptions
class OpenTSDBException(Exception):
    status = None


class IllegalDataException(OpenTSDBException):
    status = 1


class IllegalStateException(OpenTSDBException):
    status = 2


class IllegalArgumentException(OpenTSDBException, ValueError):
    status = 3


class NoSuchElementException(OpenTSDBException, KeyError):
    status = 4


class UnsupportedOperationException(OpenTSDBException):
    status = 5


class DeviceException(OpenTSDBException):
    status = 6


class CapacityException(OpenTSDBException):
    status = 7


_STATUS_EXC = {c.status: c for c in (
    IllegalDataException, IllegalStateException, IllegalArgumentException,
    NoSuchElementException, UnsupportedOperationException, DeviceException,
    CapacityException)}


def raise_for_status(status, msg=""):
    if status == 0:
        return
    raise _STATUS_EXC.get(status, OpenTSDBException)(msg)


# -------------------------------------------------------------- enums
class Interpolation(IntEnum):
    """Aggregators.Interpolation, Aggregators.java:38-44."""
    LERP = 0
    ZIM = 1
    MAX = 2
    MIN = 3
    PREV = 4


class FillPolicy(IntEnum):
    """FillPolicy.java:22-28."""
    NONE = 0
    ZERO = 1
    NOT_A_NUMBER = 2
    NULL = 3
    SCALAR = 4

    def getName(self):
        return {0: "none", 1: "zero", 2: "nan", 3: "null", 4: "scalar"}[
            int(self)]

    @staticmethod
    def fromString(name):
        for p in FillPolicy:
            if p.getName().lower() == str(name).lower():
                return p
        raise IllegalArgumentException("Unrecognized fill policy: " + name)


# -------------------------------------------------------------- aggregators
class Aggregator:
    """An entry of the Aggregators registry (Aggregator.java:26-117)."""

    def __init__(self, agg_id, name, interpolation, registry_name=None):
        self.id = agg_id
        self.name = name
        self.registry_name = registry_name or name
        self._interp = interpolation

    def interpolationMethod(self):
        return self._interp

    def __str__(self):
        return self.name

    toString = __str__

    def __repr__(self):
        return "Aggregator(%s)" % self.name


_I = Interpolation
# (id, registry key, toString, interpolation) — Aggregators.java:47-203
_AGG_TABLE = [
    (0, "sum", "sum", _I.LERP), (1, "pfsum", "pfsum", _I.PREV),
    (2, "min", "min", _I.LERP), (3, "max", "max", _I.LERP),
    (4, "avg", "avg", _I.LERP), (5, "median", "median", _I.LERP),
    (6, "none", "raw", _I.ZIM), (7, "mult", "multiply", _I.LERP),
    (8, "dev", "dev", _I.LERP), (9, "diff", "diff", _I.LERP),
    (10, "zimsum", "zimsum", _I.ZIM), (11, "mimmin", "mimmin", _I.MAX),
    (12, "mimmax", "mimmax", _I.MIN), (13, "squareSum", "squareSum", _I.ZIM),
    (14, "count", "count", _I.ZIM), (15, "first", "first", _I.ZIM),
    (16, "last", "last", _I.ZIM),
]
_PCT = ["p999", "p99", "p95", "p90", "p75", "p50"]
for _j, _n in enumerate(_PCT):
    _AGG_TABLE.append((17 + _j, _n, _n, _I.LERP))
for _j, _n in enumerate(_PCT):
    _AGG_TABLE.append((23 + _j, "e%sr3" % _n, "e%sr3" % _n, _I.LERP))
for _j, _n in enumerate(_PCT):
    _AGG_TABLE.append((29 + _j, "e%sr7" % _n, "e%sr7" % _n, _I.LERP))


class Aggregators:
    """Static registry (Aggregators.java:175-228)."""
    _by_name = {}
    _by_id = {}
    for _id, _key, _s, _ip in _AGG_TABLE:
        _a = Aggregator(_id, _s, _ip, _key)
        _by_name[_key] = _a
        _by_id[_id] = _a
    del _id, _key, _s, _ip, _a

    @classmethod
    def get(cls, name):
        a = cls._by_name.get(name)
        if a is None:
            raise NoSuchElementException("No such aggregator: " + str(name))
        return a

    @classmethod
    def set(cls):
        return set(cls._by_name.keys())

    @classmethod
    def by_id(cls, agg_id):
        return cls._by_id[agg_id]


for _key, _a in Aggregators._by_name.items():
    setattr(Aggregators, {"mult": "MULTIPLY", "squareSum": "SQUARESUM"}.get(
        _key, _key.upper()), _a)
Aggregators.NONE = Aggregators._by_name["none"]


# ---------------------------------------------------------------- DateTime
class DateTime:
    @staticmethod
    def parseDuration(duration):
        """DateTime.parseDuration, DateTime.java:187-231."""
        if not duration:
            raise IllegalArgumentException("Cannot parse null or empty duration")
        unit = 0
        while duration[unit].isdigit():
            unit += 1
            if unit >= len(duration):
                raise IllegalArgumentException(
                    "Invalid duration, must have an integer and unit: " +
                    duration)
        try:
            interval = int(duration[:unit])
        except ValueError:
            raise IllegalArgumentException("Invalid duration (number): " +
                                           duration)
        if interval <= 0:
            raise IllegalArgumentException("Zero or negative duration: " +
                                           duration)
        c = duration.lower()[-1]
        if c == "s":
            if len(duration) >= 2 and duration[-2] == "m":
                return interval
            mult = 1
        elif c == "m":
            mult = 60
        elif c == "h":
            mult = 3600
        elif c == "d":
            mult = 3600 * 24
        elif c == "w":
            mult = 3600 * 24 * 7
        elif c == "n":
            mult = 3600 * 24 * 30
        elif c == "y":
            mult = 3600 * 24 * 365
        else:
            raise IllegalArgumentException("Invalid duration (suffix): " +
                                           duration)
        mult *= 1000
        if float(interval) * mult > LONG_MAX:
            raise IllegalArgumentException(
                "Duration must be < Long.MAX_VALUE ms: " + duration)
        return interval * mult


# ------------------------------------------------- DownsamplingSpecification
class DownsamplingSpecification:
    """DownsamplingSpecification.java:116-191: "<n><unit>[c]-<agg>[-<fill>]"
    or "0all-<agg>"."""
    NO_INTERVAL = 0

    def __init__(self, specification=None, interval_ms=None, function=None,
                 fill_policy=FillPolicy.NONE):
        if specification is None and interval_ms is not None:
            # deprecated numeric ctor (interval, function, fill)
            if interval_ms <= 0:
                raise IllegalArgumentException("interval not > 0: %r" %
                                               interval_ms)
            if function is None:
                raise IllegalArgumentException("function cannot be null")
            if function is Aggregators.NONE:
                raise IllegalArgumentException(
                    "cannot use the NONE aggregator for downsampling")
            self.interval = int(interval_ms)
            self.function = function
            self.fill_policy = FillPolicy(fill_policy)
            self.string_interval = None
            self.use_calendar = False
            self.run_all = False
            self.timezone = None
            return
        if specification is None:
            raise IllegalArgumentException(
                "Downsampling specifier cannot be null")
        parts = specification.split("-")
        if len(parts) < 2:
            raise IllegalArgumentException(
                "Invalid downsampling specifier '%s': must provide at least "
                "interval and function" % specification)
        if len(parts) > 3:
            raise IllegalArgumentException(
                "Invalid downsampling specifier '%s': must consist of "
                "interval, function, and optional fill policy" % specification)
        self.run_all = False
        self.timezone = None  # DateTime.timezones.get(UTC_ID)
        if "all" in parts[0]:
            self.interval = self.NO_INTERVAL
            self.use_calendar = False
            self.string_interval = parts[0]
            self.run_all = True
        elif parts[0].endswith("c"):
            self.string_interval = parts[0][:-1]
            self.interval = DateTime.parseDuration(self.string_interval)
            self.use_calendar = True
        else:
            self.interval = DateTime.parseDuration(parts[0])
            self.use_calendar = False
            self.string_interval = parts[0]
        try:
            self.function = Aggregators.get(parts[1])
        except NoSuchElementException:
            raise IllegalArgumentException("No such downsampling function: " +
                                           parts[1])
        if self.function is Aggregators.NONE:
            raise IllegalArgumentException(
                "cannot use the NONE aggregator for downsampling")
        if len(parts) == 3:
            try:
                self.fill_policy = FillPolicy.fromString(parts[2])
            except IllegalArgumentException:
                raise IllegalArgumentException(
                    "No such fill policy: '%s'" % parts[2])
        else:
            self.fill_policy = FillPolicy.NONE

    def getInterval(self):
        return self.interval

    def getFunction(self):
        return self.function

    def getFillPolicy(self):
        return self.fill_policy

    def useCalendar(self):
        return self.use_calendar

    def setUseCalendar(self, use_calendar):
        self.use_calendar = bool(use_calendar)

    def getStringInterval(self):
        return self.string_interval

    def setTimezone(self, timezone):
        """DownsamplingSpecification.setTimezone (:202-207): a zone name or
        tzinfo."""
        if timezone is None:
            raise IllegalArgumentException("Timezone cannot be null")
        self.timezone = timezone

    def getTimezone(self):
        return self.timezone

    def calendar_interval(self):
        """(n, calendar unit) as the Downsampler ctor parses string_interval
        (Downsampler.java:131-141)."""
        from . import jcalendar
        return jcalendar.parse_calendar_interval(self.string_interval)


# -------------------------------------------------------------- RateOptions
class RateOptions:
    """RateOptions.java:27-176."""
    DEFAULT_RESET_VALUE = 0

    def __init__(self, counter=False, counter_max=LONG_MAX,
                 reset_value=DEFAULT_RESET_VALUE, drop_resets=False):
        self.counter = bool(counter)
        self.counter_max = int(counter_max)
        self.reset_value = int(reset_value)
        self.drop_resets = bool(drop_resets)

    def isCounter(self):
        return self.counter

    def getCounterMax(self):
        return self.counter_max

    def getResetValue(self):
        return self.reset_value

    def getDropResets(self):
        return self.drop_resets


# -------------------------------------------------- TsdbQuery scan bounds
def _to_seconds(t):
    return t // 1000 if (t & SECOND_MASK) != 0 else t


def get_scan_start_time_seconds(start, downsampler=None):
    """TsdbQuery.getScanStartTimeSeconds, TsdbQuery.java:1573-1612
    (no rollups).  `start` is the query start, seconds or ms."""
    start = _to_seconds(start)
    aligned = start
    if downsampler is not None and downsampler.getInterval() > 0:
        off = (1000 * start) % downsampler.getInterval()
        aligned -= off // 1000
    ts_off = aligned % MAX_TIMESPAN
    r = aligned - ts_off
    return r if r > 0 else 0


def get_scan_end_time_seconds(end, downsampler=None):
    """TsdbQuery.getScanEndTimeSeconds, TsdbQuery.java:1616-1675."""
    if (end & SECOND_MASK) != 0:
        end //= 1000
        if end == 0:
            end += 1
    if downsampler is not None and downsampler.getInterval() > 0:
        off = (1000 * end) % downsampler.getInterval()
        aligned = end + (downsampler.getInterval() - off) // 1000
        ts_off = aligned % MAX_TIMESPAN
        return aligned if ts_off == 0 else aligned + (MAX_TIMESPAN - ts_off)
    ts_off = end % MAX_TIMESPAN
    return end + (MAX_TIMESPAN - ts_off)


def to_ms(t):
    """SpanGroup ctor normalisation, SpanGroup.java:267-270."""
    return t * 1000 if (t & SECOND_MASK) == 0 else t


# ---------------------------------------------------------- query spec
def make_spec(start_time, end_time, aggregator, downsampler=None,
              query_start=0, query_end=0, rate=False, rate_options=None,
              interpolation=None, normalize=False, cal_edges=None,
              cal_cover_ms=None):
    """Builds the otsdb_query_spec of one AggregationIterator.create call
    (AggregationIterator.java:351-380).  start/end are the iterator window in
    ms; with normalize=True they are SpanGroup bounds (seconds or ms) and are
    normalised like SpanGroup.java:267-270."""
    from . import abi
    if isinstance(aggregator, str):
        aggregator = Aggregators.get(aggregator)
    if isinstance(downsampler, str):
        downsampler = DownsamplingSpecification(downsampler)
    s = abi.QuerySpec()
    s.start_ms = to_ms(int(start_time)) if normalize else int(start_time)
    s.end_ms = to_ms(int(end_time)) if normalize else int(end_time)
    s.query_start_ms = int(query_start)
    s.query_end_ms = int(query_end)
    s.agg_id = aggregator.id
    s.interp = -1 if interpolation is None else int(interpolation)
    if downsampler is not None:
        s.ds_interval_ms = int(downsampler.getInterval())
        s.ds_agg_id = downsampler.getFunction().id
        s.fill = int(downsampler.getFillPolicy())
        s.run_all = int(bool(downsampler.run_all))
        s.use_calendar = int(bool(downsampler.useCalendar()))
        if s.use_calendar and not s.run_all:
            # the query's calendar grid (opentsdb_amd/jcalendar.py); raises
            # UnsupportedOperationException when it depends on the series
            import numpy as np
            from . import jcalendar
            anchors = None
            if cal_edges is None:
                n, unit = downsampler.calendar_interval()
                tz = downsampler.getTimezone()
                try:
                    cal_edges = jcalendar.calendar_edges(
                        s.start_ms, s.end_ms, n, unit, tz,
                        cover_ms=cal_cover_ms)
                except UnsupportedOperationException:
                    # the grid depends on each series' first point: chains
                    # per anchor (otsdb_query_spec.cal_anchors)
                    cal_edges, anchors, anchor_edge = \
                        jcalendar.calendar_anchor_tables(
                            s.start_ms, s.end_ms, n, unit, tz,
                            cover_ms=cal_cover_ms)
            edges = np.ascontiguousarray(cal_edges, np.int64)
            s._cal_edges_ref = edges  # keeps the table alive with the spec
            s.cal_edges = edges.ctypes.data
            s.n_cal_edges = len(edges)
            if anchors is not None:
                a = np.ascontiguousarray(anchors, np.int64)
                ae = np.ascontiguousarray(anchor_edge, np.int64)
                s._cal_anchor_refs = (a, ae)
                s.cal_anchors = a.ctypes.data
                s.cal_anchor_edge = ae.ctypes.data
                s.n_cal_anchors = len(a)
    ro = rate_options or RateOptions()
    s.rate = int(bool(rate))
    s.counter = int(ro.counter)
    s.drop_resets = int(ro.drop_resets)
    s.counter_max = ro.counter_max
    s.reset_value = ro.reset_value
    return s
