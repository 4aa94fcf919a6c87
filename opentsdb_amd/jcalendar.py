"""Calendar downsampling grids: the bucket edges of a "<n><unit>c-<agg>"
downsampler, computed with the semantics of java.util.GregorianCalendar as
the reference drives it.

Reference:
  DateTime.previousInterval          src/utils/DateTime.java:450-610
  DateTime.unitsToCalendarType       src/utils/DateTime.java:621-645
  ValuesInInterval (calendar branch) src/core/Downsampler.java:330-345,
                                     :383-397, :422-449
  FillingDownsampler (calendar)      src/core/FillingDownsampler.java:113-135,
                                     :276-287

In OpenTSDB every series' calendar grid is anchored at
previousInterval(first point) and stepped with Calendar.add.  The engine
buckets every series of a query on ONE edge table (otsdb_query_spec.cal_edges)
so it supports exactly the queries whose grid does not depend on where a
series starts: `calendar_edges` proves that for the query window (every
"top of <period>" instant previousInterval can anchor at is an edge) and
raises UnsupportedOperationException otherwise — the reference then keeps
its own iterators.  The JNI side computes the same table with the
reference's own DateTime.previousInterval.

GregorianCalendar rules restated here (JDK 8 java.util.GregorianCalendar):
  * add(HOUR_OF_DAY | MINUTE | SECOND | MILLISECOND, n): plain millisecond
    arithmetic;
  * add(DAY_OF_MONTH, n): same wall-clock time n days later, computed with
    the old zone offset, then corrected by the offset change unless that
    moves the date;
  * add(MONTH | YEAR, n): field arithmetic, day of month pinned to the
    month's length, wall clock kept;
  * setting fields then reading the time resolves a wall-clock time in a DST
    gap with the offset before the transition and in an overlap with the
    offset after it (ZoneInfo.getOffsetsByWall);
  * weeks start on Sunday (Locale.US, as the reference's tests assume).
"""
import bisect
from datetime import date, datetime, timedelta, timezone

from .core import (IllegalArgumentException, UnsupportedOperationException)

UTC = timezone.utc
_EPOCH = datetime(1970, 1, 1)

MILLISECOND, SECOND, MINUTE, HOUR_OF_DAY, DAY_OF_MONTH, DAY_OF_WEEK, \
    MONTH, YEAR = "ms", "s", "m", "h", "d", "w", "n", "y"
_UNIT_MS = {MILLISECOND: 1, SECOND: 1000, MINUTE: 60000, HOUR_OF_DAY: 3600000}
WEEK_LENGTH = 7
MAX_EDGES = 1 << 22


def get_timezone(tz):
    """DateTime.timezones.get(name); None -> UTC."""
    if tz is None:
        return UTC
    if isinstance(tz, str):
        if tz.upper() == "UTC":
            return UTC
        from zoneinfo import ZoneInfo
        try:
            return ZoneInfo(tz)
        except Exception as e:  # noqa: BLE001
            raise IllegalArgumentException("Unknown timezone: " + tz) from e
    return tz


def units_to_calendar_type(units):
    """DateTime.unitsToCalendarType, DateTime.java:621-645."""
    if not units:
        raise IllegalArgumentException("Units cannot be null or empty")
    lc = units.lower()
    if lc in (MILLISECOND, SECOND, MINUTE, HOUR_OF_DAY, DAY_OF_MONTH,
              DAY_OF_WEEK, MONTH, YEAR):
        return lc
    raise IllegalArgumentException("Unrecognized unit type: " + units)


def parse_calendar_interval(string_interval):
    """Downsampler ctor, Downsampler.java:131-141: "<n><unit>" -> (n, unit)."""
    s = string_interval
    if "ms" in s.lower():
        return int(s[:-2]), units_to_calendar_type(s[-2:])
    return int(s[:-1]), units_to_calendar_type(s[-1:])


# ------------------------------------------------------------ wall clock
def _ms(naive_utc):
    d = naive_utc - _EPOCH
    return (d.days * 86400 + d.seconds) * 1000 + d.microseconds // 1000


def _local(t_ms, tz):
    """computeFields: the wall-clock fields of instant t_ms in tz."""
    aware = datetime.fromtimestamp(t_ms // 1000, tz).replace(
        microsecond=(t_ms % 1000) * 1000)
    return aware.replace(tzinfo=None), aware.utcoffset()


def _wall_to_ms(naive, tz):
    """computeTime: wall-clock fields -> instant (getOffsetsByWall: a gap
    resolves with the offset before the transition, an overlap with the one
    after it)."""
    oa = naive.replace(tzinfo=tz, fold=0).utcoffset()
    ob = naive.replace(tzinfo=tz, fold=1).utcoffset()
    if oa == ob:
        return _ms(naive - oa)
    ra = (naive - oa).replace(tzinfo=UTC).astimezone(tz).replace(tzinfo=None)
    rb = (naive - ob).replace(tzinfo=UTC).astimezone(tz).replace(tzinfo=None)
    off = ob if (ra == naive and rb == naive) else oa  # overlap -> after
    return _ms(naive - off)


def _days_in_month(y, m):
    if m == 12:
        return 31
    return (date(y, m + 1, 1) - date(y, m, 1)).days


def cal_add(t_ms, unit, amount, tz):
    """GregorianCalendar.add(field, amount) on a calendar at t_ms."""
    if amount == 0:
        return t_ms
    if unit in _UNIT_MS:
        return t_ms + amount * _UNIT_MS[unit]
    local, off = _local(t_ms, tz)
    if unit in (DAY_OF_MONTH, DAY_OF_WEEK):
        fd = local.date() + timedelta(days=amount)
        t = _ms(datetime.combine(fd, local.time()) - off)
        _, off2 = _local(t, tz)
        if off2 != off:
            d = off - off2
            t2 = t + (d.days * 86400 + d.seconds) * 1000 + d.microseconds // 1000
            if _local(t2, tz)[0].date() == fd:
                t = t2
        return t
    if unit == MONTH:
        m0 = local.month - 1 + amount
        y = local.year + m0 // 12
        m = m0 % 12 + 1
    elif unit == YEAR:
        y, m = local.year + amount, local.month
        if y <= 0:
            raise UnsupportedOperationException("year before the epoch")
    else:
        raise IllegalArgumentException("Unexpected unit: %r" % unit)
    day = min(local.day, _days_in_month(y, m))
    return _wall_to_ms(local.replace(year=y, month=m, day=day), tz)


def _set_fields(t_ms, tz, top):
    """setTimeInMillis(t) then set() the fields below `top` to their minimum
    (DateTime.previousInterval's snapping) and read the time back."""
    local, _ = _local(t_ms, tz)
    local = local.replace(microsecond=0)
    if top == MILLISECOND:  # top of second
        pass
    elif top == SECOND:     # top of minute
        local = local.replace(second=0)
    elif top == MINUTE:     # top of hour
        local = local.replace(second=0, minute=0)
    elif top == HOUR_OF_DAY:  # top of day
        local = local.replace(second=0, minute=0, hour=0)
    elif top == DAY_OF_MONTH:  # top of month
        local = local.replace(second=0, minute=0, hour=0, day=1)
    elif top == YEAR:       # top of year
        local = local.replace(second=0, minute=0, hour=0, day=1, month=1)
    elif top == DAY_OF_WEEK:  # Sunday of the week (WEEK_OF_MONTH+DAY_OF_WEEK)
        local = local.replace(second=0, minute=0, hour=0)
        local -= timedelta(days=(local.weekday() + 1) % 7)
    else:
        raise IllegalArgumentException("bad top %r" % top)
    return _wall_to_ms(local, tz)


def _anchor_rule(interval, unit):
    """(top, unit_override, interval_override, pre_step) of
    DateTime.previousInterval's switch, DateTime.java:468-599."""
    if unit == MILLISECOND:
        if 1000 % interval == 0:
            return MILLISECOND, unit, interval, interval > 1000
        return SECOND, unit, interval, False
    if unit == SECOND:
        if 60 % interval == 0:
            return SECOND, unit, interval, interval > 60
        return MINUTE, unit, interval, False
    if unit == MINUTE:
        if 60 % interval == 0:
            return MINUTE, unit, interval, interval > 60
        return HOUR_OF_DAY, unit, interval, False
    if unit == HOUR_OF_DAY:
        if 24 % interval == 0:
            return HOUR_OF_DAY, unit, interval, interval > 24
        return DAY_OF_MONTH, unit, interval, False
    if unit == DAY_OF_MONTH:
        if interval == 1:
            return DAY_OF_MONTH, unit, interval, False
        return YEAR, unit, interval, False
    if unit == DAY_OF_WEEK:
        # Both branches snap to a Sunday at or before ts (the current week's
        # or one in January), then step 7 days while <= ts: the result is
        # the Sunday of ts's week either way (TestDateTime.java:826-829)
        return DAY_OF_WEEK, DAY_OF_MONTH, 7, False
    if unit in (MONTH, YEAR):
        return YEAR, unit, interval, False
    raise IllegalArgumentException("Unexpected unit_overrides of type: %r"
                                   % unit)


def previous_interval(ts, interval, unit, tz=None):
    """DateTime.previousInterval(ts, interval, unit, tz), DateTime.java:450."""
    if ts < 0:
        raise IllegalArgumentException("Timestamp cannot be less than zero")
    if interval < 1:
        raise IllegalArgumentException("Interval must be greater than zero")
    tz = get_timezone(tz)
    top, u, iv, pre = _anchor_rule(interval, unit)
    c = _set_fields(ts, tz, top)
    if pre:
        c = cal_add(c, u, -iv, tz)
    if c == ts:
        return c
    while c <= ts:
        c = cal_add(c, u, iv, tz)
    return cal_add(c, u, -iv, tz)


def step(t_ms, interval, unit, tz, n=1):
    """The Downsampler's interval step (Downsampler.java:387-394)."""
    if unit == DAY_OF_WEEK:
        return cal_add(t_ms, DAY_OF_MONTH, n * interval * WEEK_LENGTH, tz)
    return cal_add(t_ms, unit, n * interval, tz)


def _tops(t0, t1, top, tz):
    """Every instant in [t0, t1] where a "top of <period>" snap can land."""
    if top in (MILLISECOND, SECOND):
        return None  # second / minute tops: checked through the offsets
    u = {MINUTE: HOUR_OF_DAY, HOUR_OF_DAY: DAY_OF_MONTH,
         DAY_OF_MONTH: MONTH, YEAR: YEAR, DAY_OF_WEEK: DAY_OF_MONTH}[top]
    n = 7 if top == DAY_OF_WEEK else 1
    t = _set_fields(t0, tz, top)
    out = []
    while t <= t1:
        if t >= t0:
            out.append(t)
        t2 = _set_fields(cal_add(t, u, n, tz), tz, top)
        if t2 <= t:  # a top that cannot advance (gap at the snap): give up
            raise UnsupportedOperationException("calendar snap does not advance")
        t = t2
    return out


def _whole_offsets(t0, t1, tz, unit_ms):
    """All zone offsets in [t0, t1] are whole multiples of unit_ms."""
    if tz is UTC:
        return True
    step_ms = 3600000
    t = t0
    while True:
        _, off = _local(t, tz)
        o = (off.days * 86400 + off.seconds) * 1000
        if o % unit_ms:
            return False
        if t >= t1:
            return True
        t = min(t + step_ms, t1)


def calendar_edges(start_ms, end_ms, interval, unit, tz=None, extra=2,
                   cover_ms=None):
    """Bucket edges of the query window [start_ms, end_ms]:
    previousInterval(start) stepped until `extra` edges past
    max(end_ms, cover_ms) — cover_ms = the batch's last point when spans hold
    points past the window (the reference's scans do not).
    Raises UnsupportedOperationException when a series starting elsewhere in
    the window would be anchored off this grid."""
    tz = get_timezone(tz)
    e = [previous_interval(start_ms, interval, unit, tz)]
    past = 0
    last = end_ms if cover_ms is None else max(end_ms, cover_ms)
    while past < extra:
        n = step(e[-1], interval, unit, tz)
        if n <= e[-1]:
            raise UnsupportedOperationException("calendar step does not advance")
        e.append(n)
        if n > last:
            past += 1
        if len(e) > MAX_EDGES:
            raise UnsupportedOperationException(
                "calendar grid too fine (> %d buckets)" % MAX_EDGES)
    top, u, iv, _ = _anchor_rule(interval, unit)
    # series' first points (after the seek) lie in [e[0], end_ms]
    t0, t1 = e[0], max(e[0], min(e[-1], end_ms))
    tops = _tops(t0, t1, top, tz)
    if tops is None:
        # second / minute tops: the grid is global iff every such top is an
        # edge, i.e. the step divides the period and the offsets are whole
        period = 1000 if top == MILLISECOND else 60000
        ms_step = iv * _UNIT_MS[u]
        if period % ms_step or not _whole_offsets(t0, t1, tz, period):
            raise UnsupportedOperationException(
                "calendar grid depends on the series' first point")
    else:
        es = set(e)
        if any(t not in es for t in tops):
            raise UnsupportedOperationException(
                "calendar grid depends on the series' first point")
    return e


SENTINEL = (1 << 63) - 1  # ends each chain of an anchored table
MAX_ANCHORS = 1 << 20


def _next_top(t, top, tz):
    """The "top of <period>" instant after top t (previousInterval's snap
    grid, DateTime.java:468-599)."""
    if top == MILLISECOND:    # top of second
        return _set_fields(t + 1000, tz, top)
    if top == SECOND:         # top of minute
        return _set_fields(t + 60000, tz, top)
    u = {MINUTE: HOUR_OF_DAY, HOUR_OF_DAY: DAY_OF_MONTH,
         DAY_OF_MONTH: MONTH, YEAR: YEAR, DAY_OF_WEEK: DAY_OF_MONTH}[top]
    n = 7 if top == DAY_OF_WEEK else 1
    t2 = _set_fields(cal_add(t, u, n, tz), tz, top)
    if t2 <= t:
        raise UnsupportedOperationException("calendar snap does not advance")
    return t2


def calendar_anchor_tables(start_ms, end_ms, interval, unit, tz=None,
                           extra=2, cover_ms=None, max_edges=MAX_EDGES,
                           max_anchors=MAX_ANCHORS):
    """Per-series calendar grids (the reference anchors every series at
    DateTime.previousInterval(its first point), Downsampler.java:330-345, and
    steps that calendar, :383-397), as the tables otsdb_query_spec carries
    when one edge table does not serve every series:

      anchors  every value previousInterval(t) takes for t in
               [start_ms, max(end_ms, cover_ms)], ascending — so
               previousInterval(t) = the largest anchor <= t;
      edges    chains, each the Downsampler's steps from an anchor until
               `extra` edges lie past max(end_ms, cover_ms), each ended by
               SENTINEL; anchors on one chain share it;
      anchor_edge[j]  index in edges of anchor j.

    Returns (edges, anchors, anchor_edge) as lists."""
    tz = get_timezone(tz)
    top, u, iv, _ = _anchor_rule(interval, unit)
    last = end_ms if cover_ms is None else max(end_ms, cover_ms)
    anchors = []
    T = _set_fields(start_ms, tz, top)
    while T <= last:
        Tn = _next_top(T, top, tz)
        # previousInterval(ts) for ts in [T, Tn): T stepped while <= ts and
        # stepped back once (DateTime.java:600-608): the chain's elements
        c = T
        while c < Tn:
            anchors.append(c)
            if len(anchors) > max_anchors:
                raise UnsupportedOperationException(
                    "calendar grid has too many anchors (> %d)" % max_anchors)
            c2 = cal_add(c, u, iv, tz)
            if c2 <= c:
                raise UnsupportedOperationException(
                    "calendar step does not advance")
            c = c2
        T = Tn
    anchors = sorted(set(anchors))
    edges, pos_of = [], {}
    anchor_edge = []
    for a in anchors:
        if a in pos_of:
            anchor_edge.append(pos_of[a])
            continue
        chain = [a]
        past = 0
        while past < extra:
            n = step(chain[-1], interval, unit, tz)
            if n <= chain[-1]:
                raise UnsupportedOperationException(
                    "calendar step does not advance")
            chain.append(n)
            if n > last:
                past += 1
        base = len(edges)
        for k, e in enumerate(chain):
            pos_of.setdefault(e, base + k)
        edges.extend(chain)
        edges.append(SENTINEL)
        if len(edges) > max_edges:
            raise UnsupportedOperationException(
                "calendar chains too long (> %d edges)" % max_edges)
        anchor_edge.append(base)
    return edges, anchors, anchor_edge


def anchored_previous_interval(tables, ts):
    """previousInterval(ts) on anchored tables: the edge index of the
    largest anchor <= ts (None before the first)."""
    edges, anchors, anchor_edge = tables
    j = bisect.bisect_right(anchors, ts) - 1
    return None if j < 0 else anchor_edge[j]


def bucket_edges_for_series(first_ts, last_ts, interval, unit, tz=None):
    """The grid ONE series follows (anchored at its first point), covering
    its points — what a lone Downsampler over that series steps through."""
    tz = get_timezone(tz)
    e = [previous_interval(first_ts, interval, unit, tz)]
    while e[-1] <= last_ts:
        e.append(step(e[-1], interval, unit, tz))
    e.append(step(e[-1], interval, unit, tz))
    return e


def edge_index(edges, t):
    """Index of the bucket [edges[k], edges[k+1]) holding t (-1 before)."""
    return bisect.bisect_right(edges, t) - 1
