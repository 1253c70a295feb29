"""CPU restatement of the disperse xlator's on-disk config guard --
TEST INFRASTRUCTURE ONLY (tests/ import it; the product never does).

Follows the reference line by line:
  pack      ec_dict_set_config   ec-helpers.c:298-330
  unpack    ec_dict_del_config   ec-helpers.c:333-380
  check     ec_config_check      ec-common.c:1151-1195
  fill      the config a create / heal stores, ec-dir-write.c:144-151,
            ec-heal.c:1268-1275
Constants: EC_CONFIG_VERSION 0, EC_CONFIG_ALGORITHM 0 (ec-common.h:22-24),
EC_GF_BITS 8 and EC_METHOD_CHUNK_SIZE 512 (ec-method.h:17-29).

Parity: the reference's tests hold no config values (tests/basic/ec/
ec-internal-xattrs.t only lists the xattr name), so this is pinned by the
bit layout itself: a 4+2 volume stores 0x0000080602000200 (version<<56 |
algorithm<<48 | gf_word_size<<40 | bricks<<32 | redundancy<<24 |
chunk_size), big-endian.
"""
import errno

EC_CONFIG_VERSION = 0
EC_CONFIG_ALGORITHM = 0
EC_GF_BITS = 8
EC_METHOD_CHUNK_SIZE = 512
U32 = 0xFFFFFFFF


def fill(bricks, redundancy):
    return dict(version=EC_CONFIG_VERSION, algorithm=EC_CONFIG_ALGORITHM,
                gf_word_size=EC_GF_BITS, bricks=bricks, redundancy=redundancy,
                chunk_size=EC_METHOD_CHUNK_SIZE)


def pack(c):
    """-> 8 bytes, or -EINVAL for a version newer than supported."""
    if c["version"] > EC_CONFIG_VERSION:
        return -errno.EINVAL
    data = (c["version"] << 56) | (c["algorithm"] << 48) | (c["gf_word_size"] << 40) | \
           (c["bricks"] << 32) | (c["redundancy"] << 24) | c["chunk_size"]
    return (data & (2**64 - 1)).to_bytes(8, "big")


def unpack(value):
    """-> dict, -EINVAL (bad length / version) or -ENODATA (all zero)."""
    if len(value) != 8:
        return -errno.EINVAL
    data = int.from_bytes(value, "big")
    if data == 0:
        return -errno.ENODATA
    version = (data >> 56) & 0xFF
    if version > EC_CONFIG_VERSION:
        return -errno.EINVAL
    return dict(version=version, algorithm=(data >> 48) & 0xFF,
                gf_word_size=(data >> 40) & 0xFF, bricks=(data >> 32) & 0xFF,
                redundancy=(data >> 24) & 0xFF, chunk_size=data & 0xFFFFFF)


def _is_power_of_2(v):          # ec-helpers.h:183-187
    return v != 0 and (v & (v - 1)) == 0


def check(nodes, redundancy, c):
    """True when ec_config_check accepts `c` for an nodes/redundancy volume;
    otherwise 'corrupted' or 'unsupported' (its two log messages)."""
    if (c["version"] == EC_CONFIG_VERSION and c["algorithm"] == EC_CONFIG_ALGORITHM and
            c["gf_word_size"] == EC_GF_BITS and c["bricks"] == nodes and
            c["redundancy"] == redundancy and c["chunk_size"] == EC_METHOD_CHUNK_SIZE):
        return True
    data_bricks = (c["bricks"] - c["redundancy"]) & U32
    if (c["redundancy"] < 1 or c["redundancy"] * 2 >= c["bricks"] or
            not _is_power_of_2(c["gf_word_size"]) or
            ((c["chunk_size"] * 8) & U32) % ((c["gf_word_size"] * data_bricks) & U32) != 0):
        return "corrupted"
    return "unsupported"
