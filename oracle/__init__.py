"""CPU oracle for the mchecksum CRC path -- TEST INFRASTRUCTURE ONLY (see crc_oracle.h)."""
