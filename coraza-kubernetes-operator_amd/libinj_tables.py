"""Authored data tables for @detectSQLi / @detectXSS.

Coraza v3.3.3 runs libinjection-go v0.2.2 (`/root/reference/go.mod:24`), a
port of libinjection 3.x.  That module -- and with it its ~9 000-entry
keyword / fingerprint table (`libinjection_sqli_data.h`) -- is not under
/root/reference and there is no network, so the tables below are AUTHORED
for this repo from the published algorithm's conventions:

* KEYWORDS: SQL words -> libinjection token type ('E' statement, 'U' union,
  'B' group/order/limit, 'k' keyword, '&' logic operator, 'o' operator,
  'f' function, 't' SQL type, 'T' T-SQL statement, 'A' collate, '1' literal,
  'v' variable-like word).  Multi-word entries are what fold's
  syntax_merge_words looks up ("UNION ALL", "ORDER BY", ...).
* TWO_CHAR_OPS: the 2-character operators parse_operator2 looks up.
* The fingerprint BLACKLIST is not a table here: it is the grammar in
  FINGERPRINT_RULES, implemented independently by the device
  (csrc/libinj.h fp_blacklisted) and the oracle (oracle/libinjection.py,
  regular expressions).  Fingerprints are upper-cased as libinjection's
  blacklist does ("v0 -> v1" conversion).

Everything that depends on these tables is PARITY UNPINNED against
libinjection-go: the GPU is checked bit-exactly against the oracle
restatement, and the reference's own KATs (coreruleset_test.go:121-127:
`1 UNION SELECT username FROM users` -> 942100, `<script>alert(1)</script>`
-> 941100, `hello world` -> pass) pin the two rules' behaviour on those
inputs.

tools/gen_libinj_tables.py writes csrc/libinj_words.h from KEYWORDS and
TWO_CHAR_OPS.
"""

KEYWORDS = {
    # statements
    "SELECT": "E", "INSERT": "E", "UPDATE": "E", "DELETE": "E", "DROP": "E",
    "CREATE": "E", "ALTER": "E", "TRUNCATE": "E", "RENAME": "E", "GRANT": "E",
    "REVOKE": "E", "CALL": "E", "SHOW": "E", "DESCRIBE": "E", "EXPLAIN": "E",
    "SET": "E", "MERGE": "E", "HANDLER": "E", "LOAD": "E", "ANALYZE": "E",
    "SELECT ALL": "E", "SELECT DISTINCT": "E", "INSERT INTO": "E",
    "DELETE FROM": "E", "REPLACE INTO": "E", "WAITFOR": "E", "WAITFOR DELAY": "E",
    "WAITFOR TIME": "E", "LOAD DATA": "E", "DROP TABLE": "E", "DROP DATABASE": "E",
    "CREATE TABLE": "E", "ALTER TABLE": "E", "USE": "E",
    # union family
    "UNION": "U", "UNION ALL": "U", "UNION DISTINCT": "U", "INTERSECT": "U",
    "EXCEPT": "U", "MINUS": "U",
    # grouping / ordering / limits
    "GROUP BY": "B", "ORDER BY": "B", "HAVING": "B", "LIMIT": "B", "OFFSET": "B",
    "PROCEDURE ANALYSE": "B",
    # keywords
    "FROM": "k", "WHERE": "k", "INTO": "k", "INTO OUTFILE": "k", "INTO DUMPFILE": "k",
    "TABLE": "k", "AS": "k", "ON": "k", "JOIN": "k", "LEFT JOIN": "k",
    "RIGHT JOIN": "k", "INNER JOIN": "k", "CROSS JOIN": "k", "NATURAL JOIN": "k",
    "OUTER JOIN": "k", "LEFT OUTER JOIN": "k", "RIGHT OUTER JOIN": "k",
    "FULL OUTER JOIN": "k", "STRAIGHT_JOIN": "k", "VALUES": "k", "VALUE": "k",
    "IN": "k", "NOT IN": "k", "CASE": "E", "WHEN": "k", "THEN": "k", "ELSE": "k",
    "END": "k", "IF EXISTS": "k", "IF NOT EXISTS": "k", "ALL": "k", "DISTINCT": "k",
    "ASC": "k", "DESC": "k", "TOP": "k", "INDEX": "k", "KEY": "k", "PRIMARY": "k",
    "FOREIGN": "k", "REFERENCES": "k", "PROCEDURE": "k", "FUNCTION": "k",
    "TRIGGER": "k", "VIEW": "k", "USING": "k", "OUTFILE": "k", "DUMPFILE": "k",
    "SCHEMA": "k", "COLUMN": "k", "DUAL": "k", "CHARACTER SET": "k",
    "FOR UPDATE": "k", "LOCK IN SHARE MODE": "k", "SHARE MODE": "k", "ESCAPE": "k",
    "WITH": "k", "ROLLUP": "k", "WITH ROLLUP": "k", "INFILE": "k", "TO": "k",
    "DATABASE": "n", "PASSWORD": "n", "USER": "n", "CURRENT_USER": "v",
    "CURRENT_DATE": "v", "CURRENT_TIME": "v", "CURRENT_TIMESTAMP": "v",
    "LOCALTIME": "v", "LOCALTIMESTAMP": "v", "USER_ID": "n", "USER_NAME": "n",
    # logic operators
    "AND": "&", "OR": "&", "XOR": "&",
    # operators
    "LIKE": "o", "NOT LIKE": "o", "RLIKE": "o", "NOT RLIKE": "o", "REGEXP": "o",
    "NOT REGEXP": "o", "SOUNDS LIKE": "o", "BETWEEN": "o", "NOT BETWEEN": "o",
    "IS": "o", "IS NOT": "o", "DIV": "o", "MOD": "o", "NOT": "o", "ILIKE": "o",
    "SIMILAR TO": "o", "GLOB": "o", "MATCH": "o", "AGAINST": "o",
    # collate
    "COLLATE": "A",
    # literals
    "NULL": "1", "TRUE": "1", "FALSE": "1", "UNKNOWN": "1",
    # functions
    "ABS": "f", "ASCII": "f", "BENCHMARK": "f", "BIN": "f", "CAST": "f",
    "CEIL": "f", "CEILING": "f", "CHAR": "f", "CHR": "f", "CHAR_LENGTH": "f",
    "CHARACTER_LENGTH": "f", "COALESCE": "f", "CONCAT": "f", "CONCAT_WS": "f",
    "CONVERT": "f", "COUNT": "f", "CURDATE": "f", "CURTIME": "f", "ELT": "f",
    "EXISTS": "f", "EXTRACTVALUE": "f", "FLOOR": "f", "GROUP_CONCAT": "f",
    "HEX": "f", "IF": "f", "IFNULL": "f", "INSTR": "f", "ISNULL": "f",
    "LCASE": "f", "LENGTH": "f", "LOAD_FILE": "f", "LOCATE": "f", "LOWER": "f",
    "LPAD": "f", "LTRIM": "f", "MAKE_SET": "f", "MAX": "f", "MD5": "f", "MID": "f",
    "MIN": "f", "NAME_CONST": "f", "NOW": "f", "NULLIF": "f", "OCT": "f",
    "ORD": "f", "PG_SLEEP": "f", "POSITION": "f", "POW": "f", "POWER": "f",
    "RAND": "f", "REPEAT": "f", "REPLACE": "f", "REVERSE": "f", "ROUND": "f",
    "RPAD": "f", "RTRIM": "f", "SHA1": "f", "SHA2": "f", "SLEEP": "f",
    "SPACE": "f", "SQRT": "f", "STRCMP": "f", "SUBSTR": "f", "SUBSTRING": "f",
    "SUBSTRING_INDEX": "f", "SUM": "f", "SYSTEM_USER": "f", "SESSION_USER": "f",
    "TRIM": "f", "UCASE": "f", "UNHEX": "f", "UPDATEXML": "f", "UPPER": "f",
    "UUID": "f", "VERSION": "f", "EXP": "f", "JSON_KEYS": "f", "GTID_SUBSET": "f",
    "XP_CMDSHELL": "f", "SP_EXECUTESQL": "f", "OPENROWSET": "f", "OPENQUERY": "f",
    "DBMS_PIPE.RECEIVE_MESSAGE": "f", "UTL_INADDR.GET_HOST_ADDRESS": "f",
    "UTL_HTTP.REQUEST": "f", "SUSER_NAME": "f", "DB_NAME": "f", "HOST_NAME": "f",
    "LEFT": "f", "RIGHT": "f", "ANY": "f", "SOME": "f", "AVG": "f",
    "TO_CHAR": "f", "TO_NUMBER": "f", "NVL": "f", "DECODE": "f", "RANDOMBLOB": "f",
    "SQLITE_VERSION": "f", "LIKELIHOOD": "f", "INET_NTOA": "f", "CONNECTION_ID": "f",
    # SQL types
    "INT": "t", "INTEGER": "t", "BIGINT": "t", "SMALLINT": "t", "TINYINT": "t",
    "VARCHAR": "t", "NVARCHAR": "t", "TEXT": "t", "DATETIME": "t", "TIMESTAMP": "t",
    "FLOAT": "t", "DOUBLE": "t", "DECIMAL": "t", "NUMERIC": "t", "REAL": "t",
    "BOOLEAN": "t", "BOOL": "t", "SIGNED": "t", "UNSIGNED": "t", "BINARY": "t",
    "VARBINARY": "t", "BLOB": "t", "NCHAR": "t",
    # T-SQL statements
    "EXEC": "T", "EXECUTE": "T", "DECLARE": "T", "SHUTDOWN": "T", "GOTO": "T",
    "PRINT": "T", "BEGIN": "T", "WHILE": "T", "RAISERROR": "T",
}

# parse_operator2's two-character operators ('&' for the logic ones)
TWO_CHAR_OPS = {
    "!!": "o", "!<": "o", "!=": "o", "!>": "o", "!~": "o", "%=": "o", "&&": "&",
    "&=": "o", "*=": "o", "+=": "o", "-=": "o", "/=": "o", "::": "o", ":=": "o",
    "<<": "o", "<=": "o", "<>": "o", "<@": "o", ">=": "o", ">>": "o", "@>": "o",
    "^=": "o", "|/": "o", "|=": "o", "||": "&", "~*": "o",
}

# Fingerprint blacklist grammar (upper-cased fingerprint f, 1..5 tokens).
# A fingerprint is blacklisted iff one of these holds ("value" = 1 S N V):
#   R1  f == "X"                              (unparsable: nested / MySQL conditional comment)
#   R2  f contains "UE" or "U(E"              (UNION [ALL] SELECT)
#   R3  f contains ";E" or ";T"               (stacked statement)
#   R4  ^[1S] )* [&O] (* [1SVF]              (tautology / comparison after a value)
#   R5  ^N )* & (* [1SVF]                     (bareword AND/OR value)
#   R6  ^[1SN] C $                            (value then comment; whitelist refines)
#   R7  ^E (* [1SVF]  |  ^E .{0,2} K  |  ^E [1SNV] ,     (SELECT expressions)
#   R8  ^[1SN] )* B [1NS(]                    (ORDER/GROUP BY n)
#   R9  ^[1SN] )+ [&O;U]                      (closing parentheses then operator)
#   R10 ^& (* [1SVF]                          (leading AND/OR)
#   R11 ^T [N1SVF(]                           (T-SQL statement)
#   R12 ^[1SN] )* U                           (value then UNION)
#   R13 ^[1SN] K [S1]                         (INTO OUTFILE 'x' ...; whitelist refines)
#   R14 ^F ( [1SNV]? )                        (function call alone: sleep(5))
FINGERPRINT_RULES = [
    ("R1", r"^X$"),
    ("R2", r"U\(?E"),
    ("R3", r";[ET]"),
    ("R4", r"^[1S]\)*[&O]\(*[1SVF]"),
    ("R5", r"^N\)*&\(*[1SVF]"),
    ("R6", r"^[1SN]C$"),
    ("R7", r"^E\(*[1SVF]|^E.{0,2}K|^E[1SNV],"),
    ("R8", r"^[1SN]\)*B[1NS(]"),
    ("R9", r"^[1SN]\)+[&O;U]"),
    ("R10", r"^&\(*[1SVF]"),
    ("R11", r"^T[N1SVF(]"),
    ("R12", r"^[1SN]\)*U"),
    ("R13", r"^[1SN]K[S1]"),
    ("R14", r"^F\([1SNV]?\)"),
]

# libinjection_xss.c BLACKTAG / BLACKATTR (the published lists)
XSS_BLACK_TAGS = [
    "APPLET", "BASE", "COMMENT", "EMBED", "FRAME", "FRAMESET", "HANDLER", "IFRAME",
    "IMPORT", "ISINDEX", "LINK", "LISTENER", "META", "NOSCRIPT", "OBJECT", "SCRIPT",
    "STYLE", "VMLFRAME", "XML", "XSS",
]
# attribute -> type: 1 black, 2 URL, 3 style, 4 indirect
XSS_BLACK_ATTRS = [
    ("ACTION", 2), ("ATTRIBUTENAME", 4), ("BY", 2), ("BACKGROUND", 2),
    ("DATAFORMATAS", 1), ("DATASRC", 1), ("DYNSRC", 2), ("FILTER", 3),
    ("FORMACTION", 2), ("FOLDER", 2), ("FROM", 2), ("HANDLER", 2), ("HREF", 2),
    ("LOWSRC", 2), ("POSTER", 2), ("SRC", 2), ("STYLE", 3), ("TO", 2),
    ("VALUES", 2), ("XLINK:HREF", 2),
]


def word_table():
    """Sorted (word, type) pairs: the keyword table plus the 2-char operators."""
    t = dict(KEYWORDS)
    t.update(TWO_CHAR_OPS)
    return sorted(t.items())
