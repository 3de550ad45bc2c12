"""CPU checks of the FilesystemStore mirror (zarrs_filesystem/src/lib.rs:173-179 key_to_fspath;
missing key -> None, :339-343) and of the file-range ABI struct (no GPU calls)."""
import ctypes as C


def test_key_to_fspath_and_get(tmp_path):
    from zarrs_amd import FilesystemStore
    st = FilesystemStore(tmp_path)
    assert st.key_to_fspath("c/0/1") == str(tmp_path / "c" / "0" / "1")
    assert st.key_to_fspath("/c/0/1") == str(tmp_path / "c" / "0" / "1")  # leading '/' stripped
    assert st.key_to_fspath("") == str(tmp_path)
    st["c/0/1"] = b"abc"
    assert st.get("c/0/1") == b"abc" and "c/0/1" in st
    assert st.get("c/9/9") is None and "c/9/9" not in st
    assert st.get("c/0/1/x") is None  # a path through a file is a missing key, not an error


def test_file_range_struct_matches_header():
    from zarrs_amd import _lib as L
    assert C.sizeof(L.FileRange) == 24
    assert L.FileRange.offset.offset == 8 and L.FileRange.len.offset == 16
    assert L.WHOLE == 2**64 - 1
    assert L.STATUS_NAMES[L.STORAGE_ERROR] == "STORAGE_ERROR"
