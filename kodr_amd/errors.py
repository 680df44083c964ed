"""kodr's sentinel errors (errors.go:5-18) as exception classes.

Status codes 1..12 of the C ABI map to these classes in the order of
errors.go:6-17; Go's ``errors.Is(err, kodr.ErrX)`` becomes
``isinstance(e, kodr_amd.errors.ErrX)`` / ``pytest.raises(ErrX)``.
"""


class KodrError(Exception):
    code = 0


class ErrCannotInvertGf256AdditiveIndentity(KodrError):
    code = 1


class ErrMatrixDimensionMismatch(KodrError):
    code = 2


class ErrAllUsefulPiecesReceived(KodrError):
    code = 3


class ErrMoreUsefulPiecesRequired(KodrError):
    code = 4


class ErrCopyFailedDuringPieceConstruction(KodrError):
    code = 5


class ErrPieceCountMoreThanTotalBytes(KodrError):
    code = 6


class ErrZeroPieceSize(KodrError):
    code = 7


class ErrBadPieceCount(KodrError):
    code = 8


class ErrCodedDataLengthMismatch(KodrError):
    code = 9


class ErrCodingVectorLengthMismatch(KodrError):
    code = 10


class ErrPieceNotDecodedYet(KodrError):
    code = 11


class ErrPieceOutOfBound(KodrError):
    code = 12


class EngineError(RuntimeError):
    """Negative status: invalid argument, OOM, HIP failure or no device."""

    def __init__(self, code, msg):
        super().__init__(f"kodr_amd engine error {code}: {msg}")
        self.code = code


BY_CODE = {c.code: c for c in KodrError.__subclasses__()}
# short names as they appear in tests/golden (Go identifiers)
BY_NAME = {c.__name__: c for c in KodrError.__subclasses__()}


def check(status):
    """Raise the exception for a C-ABI status code (0 = OK)."""
    if status == 0:
        return
    if status in BY_CODE:
        from ._lib import lib
        raise BY_CODE[status](lib().rlnc_status_string(status).decode())
    from ._lib import lib
    raise EngineError(status, (lib().rlnc_status_string(status) or b"").decode() + ": "
                      + (lib().rlnc_last_hip_error() or b"").decode())
