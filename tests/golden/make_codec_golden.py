"""Generates tests/golden/codec_golden.npz with the REFERENCE's own wire codec
(oracle/_ref/libppref_json.so: helpers.h hasData + nlohmann json.hpp compiled from /root/reference,
glue restating src/main.cpp:1217-1252, 1325-1333, 1461-1464): the telemetry corpus of
tests/codec_corpus.py with the values the reference reads from each frame, and control messages
dumped for a value corpus. Run from the repo root after `make -C oracle`."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import codec_corpus  # noqa: E402
import oracle_lib  # noqa: E402


def main():
    rj = oracle_lib.load_ref_json()
    assert rj is not None, "oracle/_ref/libppref_json.so not built"
    msgs = codec_corpus.corpus(2024, 400)
    st, ego, px, py, npv, ncar, ids, cars = [], [], [], [], [], [], [], []
    for m in msgs:
        s, e, a, b, n, i, c = oracle_lib.ref_json_parse(rj, m)
        st.append(s); ego.append(e); px.append(a); py.append(b); npv.append(n); ncar.append(len(i))
        ii = np.zeros(16, np.int32); cc = np.zeros((16, 4)); ii[:len(i)] = i[:16]; cc[:len(i)] = c[:16]
        ids.append(ii); cars.append(cc)
    vals = codec_corpus.control_values(7, 64)
    dumps = [oracle_lib.ref_json_dump(rj, vals[k:k + 50], vals[::-1][k:k + 50]) for k in range(0, len(vals) - 50, 7)]
    buf = b"".join(msgs)
    off = np.cumsum([0] + [len(m) for m in msgs])
    dbuf = b"".join(dumps)
    doff = np.cumsum([0] + [len(d) for d in dumps])
    # simulator-shaped frames the GPU codec parses itself, and planner-like control dumps it formats
    # itself: the reference's fields / bytes for the device codec's direct parity test
    smsgs = codec_corpus.sim_corpus(2025, 512)
    sst, sego, spx, spy, snpv, sids, scars = [], [], [], [], [], [], []
    for m in smsgs:
        s, e, a, b, n, i, c = oracle_lib.ref_json_parse(rj, m)
        assert s != 0 or len(i) == 12
        sst.append(s); sego.append(e); spx.append(a); spy.append(b); snpv.append(n)
        ii = np.zeros(12, np.int32); cc = np.zeros((12, 4)); ii[:len(i)] = i; cc[:len(i)] = c
        sids.append(ii); scars.append(cc)
    txs, tys, tn = codec_corpus.trajectory_values(2026, 50, 96)
    tdumps = [oracle_lib.ref_json_dump(rj, txs[:tn[k], k], tys[:tn[k], k]) for k in range(len(tn))]
    sbuf = b"".join(smsgs)
    soff = np.cumsum([0] + [len(m) for m in smsgs])
    tbuf = b"".join(tdumps)
    toff = np.cumsum([0] + [len(d) for d in tdumps])
    np.savez_compressed(os.path.join(HERE, "codec_golden.npz"),
                        sim_buf=np.frombuffer(sbuf, np.uint8), sim_off=soff, sim_status=np.array(sst, np.int32),
                        sim_ego=np.array(sego), sim_prev_x=np.array(spx), sim_prev_y=np.array(spy),
                        sim_n_prev=np.array(snpv, np.int32), sim_car_id=np.array(sids), sim_cars=np.array(scars),
                        traj_x=txs, traj_y=tys, traj_n=tn, traj_buf=np.frombuffer(tbuf, np.uint8), traj_off=toff,
                        msg_buf=np.frombuffer(buf, np.uint8), msg_off=off, status=np.array(st, np.int32),
                        ego=np.array(ego), prev_x=np.array(px), prev_y=np.array(py), n_prev=np.array(npv, np.int32),
                        n_cars=np.array(ncar, np.int32), car_id=np.array(ids), cars=np.array(cars),
                        values=vals, dump_buf=np.frombuffer(dbuf, np.uint8), dump_off=doff)
    print(f"{len(msgs)} frames ({int(np.sum(np.array(st) == 0))} telemetry), {len(dumps)} control messages; "
          f"{len(smsgs)} simulator-shaped frames, {len(tdumps)} trajectory dumps")


if __name__ == "__main__":
    main()
