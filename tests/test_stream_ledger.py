"""StreamLedger (models/decoder.py): the fork / join bookkeeping that every comm-stream schedule goes through.
A fork left open must fail the forward on the host - before a HIP graph capture could end with unjoined work -
and waiting on a mark joins that fork and every earlier one (the comm stream runs in order). CPU only."""
import pytest

from llmss_amd.models.decoder import StreamLedger


def test_join_clears_every_fork():
    led = StreamLedger()
    for _ in range(3):
        led.fork(None, None)
    assert led.open == [1, 2, 3] and led.forks == 3
    led.join(None, None)
    assert not led.open
    led.check("ok")


def test_wait_on_a_mark_joins_it_and_the_earlier_forks():
    led = StreamLedger()
    a = led.mark(None, led.fork(None, None))
    b = led.mark(None, led.fork(None, None))
    c = led.mark(None, led.fork(None, None))
    led.wait(None, b)
    assert led.open == [3]
    led.wait(None, a)  # already covered: no effect
    assert led.open == [3]
    led.wait(None, c)
    led.check("ok")


def test_unjoined_fork_fails_the_forward():
    led = StreamLedger()
    led.fork(None, None)
    with pytest.raises(RuntimeError, match="never joined"):
        led.check("DecoderLM.hidden_states")
    led.check("reset after the error")  # the failed forward does not poison the next one


def test_schedule_ab_times_three_representative_buckets():
    """The capture-time schedule A/B times the largest candidate bucket, the largest at most half of it and the
    smallest (engine start-up at TP=8); the rest adopt the nearest timed bucket's winner."""
    from llmss_amd.engine.engine import LLMEngine

    big = [64, 96, 128, 160, 192, 224, 256, 288, 320, 352, 384, 416, 448, 480, 512]
    assert LLMEngine._ab_buckets(big) == [64, 256, 512]
    assert LLMEngine._ab_buckets([16, 24]) == [16, 24]
    assert LLMEngine._ab_buckets([8, 16, 24]) == [8, 24]
    assert LLMEngine._ab_buckets([128]) == [128]
    assert LLMEngine._ab_buckets([]) == []
