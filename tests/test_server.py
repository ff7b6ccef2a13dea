"""Simulator shim: pp_serve speaks the reference's uWS side of the wire
(src/main.cpp:1214-1494). CPU tests cover the protocol (handshake known answer, manual / ignored
frames, ping, fragmentation, close, several clients); the GPU tests drive closed-loop episodes
through the socket and check every control message against the restatement's plan."""
import ctypes as C
import socket
import time

import numpy as np
import pytest

import oracle_lib
from oracle_lib import ppamd
from ppamd.wsclient import WSClient

MANUAL = b'42["manual",{}]'


@pytest.fixture(scope="module")
def m():
    return ppamd.Map(*oracle_lib.highway_map())


def test_accept_key_known_answer():
    out = C.create_string_buffer(64)
    assert ppamd.lib.pp_ws_accept_key(b"dGhlIHNhbXBsZSBub25jZQ==", out, 64) == 0   # RFC 6455 §1.3
    assert out.value == b"s3pPLMBiTxaQ9kYGzzhZRbK+xOo="


def test_protocol_without_telemetry(m):
    srv = ppamd.Server(m, max_clients=8)
    try:
        a, b = WSClient(srv.port.value), WSClient(srv.port.value)
        assert a.status_line.startswith(b"HTTP/1.1 101") and a.accept_ok and b.accept_ok
        a.send(b"2")                                    # engine.io ping text: no answer (not "42")
        a.send(b'42["other",{"x":1}]')                  # another event: no answer
        a.send(b'42["telemetry",null]')                 # no data: manual
        assert a.recv() == MANUAL
        b.send_frame(b'42["telemetry",', opcode=1, fin=False)   # fragmented message
        b.send_frame(b"null]", opcode=0, fin=True)
        assert b.recv() == MANUAL
        a.send_frame(b"hello", opcode=9)                # ping -> pong with the same payload
        assert a.recv_frame() == (10, b"hello")
        b.send(b'42["manual",{}]')                      # another event from the client: ignored
        for _ in range(5):
            b.send(b'42["telemetry",null]')
        for _ in range(5):
            assert b.recv() == MANUAL
        a.close()
        b.close()
        # a plain HTTP request without the upgrade key is refused
        s = socket.create_connection(("127.0.0.1", srv.port.value), timeout=5)
        s.sendall(b"GET / HTTP/1.1\r\nHost: x\r\n\r\n")
        assert s.recv(100).startswith(b"HTTP/1.1 400")
        s.close()
    finally:
        rc, stats = srv.close()
    assert rc == 0 and stats[0] == 0 and stats[2] >= 3 and stats[3] >= 7


def episode_frames(olib, wx, wy, F, first_scene, id_of=lambda j: j):
    """Telemetry frames of a closed-loop episode from the restatement (one scene), rendered as
    the simulator would send them (car j reported with id id_of(j), an increasing map), with the
    restatement's plan for each."""
    sc, tr = ppamd.synth_traffic_host(ppamd.Map(wx, wy), 1, seed=0x5EED0007, first=first_scene)
    sc["prev_target_lane"][:] = 1           # the lambda's target_lane starts at 1 (src/main.cpp:1195)
    prm = ppamd.default_params(n_speeds=1)
    frames, plans = [], []
    for f in range(F):
        tel = {k: v.copy() for k, v in sc.items()}
        lg = oracle_lib.oracle_rollout(olib, wx, wy, sc, tr, prm, 1, 3, 120.0)
        n = int(lg["n_out"][0, 0])
        plans.append((lg["plan_x"][0, :n, 0], lg["plan_y"][0, :n, 0]))
        npv = min(int(tel["n_prev"][0]), 10)
        fmt = lambda a: ",".join(repr(float(v)) for v in a)
        rows = ",".join("[%d,%r,%r,%r,%r,0,0]" % (id_of(int(tel["car_id"][j, 0])), float(tel["car_x"][j, 0]),
                                                   float(tel["car_y"][j, 0]), float(tel["car_vx"][j, 0]),
                                                   float(tel["car_vy"][j, 0])) for j in range(int(tel["n_cars"][0])))
        frames.append(('42["telemetry",{"x":%r,"y":%r,"yaw":%r,"speed":%r,"s":0,"d":0,"previous_path_x":[%s],'
                       '"previous_path_y":[%s],"end_path_s":0,"end_path_d":0,"sensor_fusion":[%s]}]'
                       % (float(tel["ego_x"][0]), float(tel["ego_y"][0]), float(tel["ego_yaw_deg"][0]),
                          float(tel["ego_speed_mph"][0]), fmt(tel["prev_x"][:npv, 0]), fmt(tel["prev_y"][:npv, 0]),
                          rows)).encode())
    return frames, plans


@pytest.mark.gpu
@pytest.mark.parametrize("id_of", [lambda j: j, lambda j: 1000 + 37 * j], ids=["ids0-11", "ids1000+"])
def test_served_episodes_match_restatement(m, id_of):
    """Four simulators in parallel, 60 frames each: every reply equals the restatement's plan of
    that frame within 1e-6 m (the car table and target lane persist per connection). With ids
    1000 + 37 j the connection's std::map holds ids far beyond the table's slot count: the plans
    are the same (the reference orders cars by id and compares ids, nothing else)."""
    wx, wy = oracle_lib.highway_map()
    olib = oracle_lib.load_oracle()
    K, F = 4, 60
    eps = [episode_frames(olib, wx, wy, F, k, id_of) for k in range(K)]
    srv = ppamd.Server(m, max_clients=K)
    try:
        cl = [WSClient(srv.port.value) for _ in range(K)]
        for f in range(F):
            for k in range(K):
                cl[k].send(eps[k][0][f])
            for k in range(K):
                msg = cl[k].recv()
                body = msg[len(b'42["control",'):-1]
                xs = np.array([float(v) for v in body[body.index(b"[") + 1:body.index(b"]")].split(b",") if v])
                ys = np.array([float(v) for v in body[body.rindex(b"[") + 1:body.rindex(b"]")].split(b",") if v])
                px, py = eps[k][1][f]
                assert len(xs) == len(px) and len(ys) == len(py), (k, f)
                # %.15g in the message: compare at its resolution
                assert np.abs(xs - px).max(initial=0) <= 1e-6 and np.abs(ys - py).max(initial=0) <= 1e-6, (k, f)
        for c in cl:
            c.close()
    finally:
        rc, stats = srv.close()
    assert rc == 0 and stats[0] == K * F
