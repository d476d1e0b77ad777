"""DAP framing on the hot path vs the reference's own hex KATs
(/root/reference/messages/src/lib.rs:4184-4340, copied here as data)."""
from janus_amd.messages import (HpkeCiphertext, PingPongMessage, PrepareError, PrepareInit, PrepareResp,
                                PrepareStepResult, ReportMetadata, ReportShare)

# roundtrip_prepare_init, case 1 (messages/src/lib.rs:4186-4241)
PI1 = ("0102030405060708090A0B0C0D0E0F10" "000000000000D431" "00000000" ""
       "2A" "0006" "303132333435" "00000006" "353433323130"
       "0000000b" "00" "00000006" "303132333435")
# case 2 (:4242-4298)
PI2 = ("100F0E0D0C0B0A090807060504030201" "0000000000011F46" "00000004" "30313233"
       "0D" "0004" "61626365" "00000004" "61626664"
       "00000005" "02" "00000000" "")
# roundtrip_prepare_resp (:4304-4340)
PR1 = ("0102030405060708090A0B0C0D0E0F10" "00" "00000013" "01" "00000006" "303132333435" "00000004" "36373839")
PR2 = "100F0E0D0C0B0A090807060504030201" "01"


def test_prepare_init_kats():
    pi1 = PrepareInit(ReportShare(ReportMetadata(bytes(range(1, 17)), 54321), b"",
                                  HpkeCiphertext(42, b"012345", b"543210")),
                      PingPongMessage.initialize(b"012345"))
    assert pi1.encode().hex().upper() == PI1.upper()
    assert PrepareInit.decode(bytes.fromhex(PI1)) == pi1
    pi2 = PrepareInit(ReportShare(ReportMetadata(bytes(range(16, 0, -1)), 73542), b"0123",
                                  HpkeCiphertext(13, b"abce", b"abfd")),
                      PingPongMessage.finish(b""))
    assert pi2.encode().hex().upper() == PI2.upper()
    assert PrepareInit.decode(bytes.fromhex(PI2)) == pi2


def test_prepare_resp_kats():
    r1 = PrepareResp(bytes(range(1, 17)),
                     PrepareStepResult(0, message=PingPongMessage(1, prep_msg=b"012345", prep_share=b"6789")))
    assert r1.encode().hex().upper() == PR1.upper()
    assert PrepareResp.decode(bytes.fromhex(PR1)) == r1
    r2 = PrepareResp(bytes(range(16, 0, -1)), PrepareStepResult(1))
    assert r2.encode().hex().upper() == PR2.upper()
    rej = PrepareResp(bytes(16), PrepareStepResult(2, error=PrepareError.VdafPrepError))
    assert rej.encode().hex() == "00" * 16 + "02" + "05"
    assert PrepareResp.decode(rej.encode()) == rej


def test_finish_message_shape():
    # helper's outbound Finish{prep_msg} for a joint-rand Prio3: 0x02 || u32 len || 16-byte seed
    m = PingPongMessage.finish(bytes(range(16)))
    assert m.encode() == b"\x02" + (16).to_bytes(4, "big") + bytes(range(16))
    assert PingPongMessage.decode(m.encode()) == m


def test_plaintext_input_share_codec():
    import pytest

    from janus_amd.messages import (EXTENSION_TASKPROV, EXTENSION_TBD, CodecError, Extension,
                                    PlaintextInputShare)
    p = PlaintextInputShare((Extension(EXTENSION_TBD, b"ab"), Extension(EXTENSION_TASKPROV)), b"\x01" * 48)
    enc = p.encode()
    assert enc[:2] == (4 + 2 + 4).to_bytes(2, "big")
    assert PlaintextInputShare.decode(enc) == p
    assert PlaintextInputShare.decode(PlaintextInputShare((), b"xyz").encode()).payload == b"xyz"
    with pytest.raises(CodecError):
        PlaintextInputShare.decode(enc + b"\x00")  # trailing bytes
    with pytest.raises(CodecError):  # unknown extension type
        PlaintextInputShare.decode((6).to_bytes(2, "big") + b"\x12\x34\x00\x00\x00\x00" + (0).to_bytes(4, "big"))
