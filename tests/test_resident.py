"""CPU tests of envs/resident.py: at most one step server per device is resident; claiming a
device for another server stops the previous one, exactly once, and releasing only forgets
the server that holds the device."""
import threading


class _FakeServer:
    def __init__(self):
        self.stops = 0

    def stop(self):
        self.stops += 1


def test_claim_stops_the_previous_server_once_per_switch():
    from gym_supplychain_amd.envs import resident
    a, b, c = _FakeServer(), _FakeServer(), _FakeServer()
    dev = 1000  # a device index no real server uses
    resident.claim(dev, a)
    resident.claim(dev, a)  # the resident server again: nothing stops
    assert a.stops == 0
    resident.claim(dev, b)
    assert a.stops == 1 and b.stops == 0
    resident.claim(dev + 1, c)  # another device: independent
    assert b.stops == 0 and c.stops == 0
    resident.release(dev, a)  # not the holder: no effect
    resident.claim(dev, b)
    assert b.stops == 0
    resident.release(dev, b)
    resident.claim(dev, a)  # the device was free: nothing to stop
    assert a.stops == 1 and b.stops == 0
    resident.release(dev, a)
    resident.release(dev + 1, c)


def test_claims_from_threads_keep_one_resident_server():
    from gym_supplychain_amd.envs import resident
    dev = 2000
    servers = [_FakeServer() for _ in range(4)]
    n = 500

    def run(s):
        for _ in range(n):
            resident.claim(dev, s)

    threads = [threading.Thread(target=run, args=(s,)) for s in servers]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    holder = resident._RESIDENT[dev]
    assert holder in servers
    # a stop happens only when a claim replaces another server: never more than the claims
    assert sum(s.stops for s in servers) <= 4 * n - 1
    resident.release(dev, holder)
    assert dev not in resident._RESIDENT
