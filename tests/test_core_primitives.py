"""Core primitives of the native runtime: latency histogram accuracy, event-loop timer
ordering/cancellation and cross-thread posts, the SPSC span ring."""
import random


def test_histogram_relative_error(native):
    rng = random.Random(7)
    values = [int(rng.lognormvariate(10, 1.5)) for _ in range(20000)]
    ps = [50, 90, 99, 99.9]
    got = native.histogram_percentiles(values, ps)
    s = sorted(values)
    for p, g in zip(ps, got):
        exact = s[min(len(s) - 1, int(p / 100 * len(s)))]
        assert abs(g - exact) <= max(2, 0.02 * exact), (p, g, exact)


def test_histogram_small_values_exact(native):
    assert native.histogram_percentiles([1, 2, 3, 4, 5], [0, 60, 100]) == [1, 3, 5]


def test_event_loop_timer_order_and_cancel(native):
    order = native.loop_timer_order([30, 10, 20, 10], cancel=[2])
    assert order[0] == -1  # posted task runs before timers fire
    assert order[1:] == [1, 3, 0]  # deadline order, FIFO for equal deadlines, #2 cancelled


def test_span_ring_bounded_and_ordered(native):
    ok, drained = native.span_ring(8, 20)
    assert ok == 8 and drained == 8  # the ring drops (and the tracer counts) the rest
    ok, drained = native.span_ring(1024, 1000)
    assert ok == drained == 1000
