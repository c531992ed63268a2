"""Insert the authored paranoia-level 2-4 rules into rulesets/crs/*.conf.

CRS v4.23.0 itself is a download (reference Makefile:185-206), unavailable
offline; the PL1 files under rulesets/crs/ are CRS-shaped stand-ins.  This
script adds CRS-shaped PL2/PL3/PL4 detection rules (ids, targets,
transformations and scoring follow CRS v4's conventions) into the existing
paranoia-gated regions, so the C4 configuration (blocking paranoia level 4)
evaluates a realistically larger rule set.  Idempotent: rules already present
(by id) are skipped.

    python tools/add_crs_pl234.py && python tools/build_crs_pl1.py
"""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CRS = os.path.join(ROOT, "rulesets", "crs")

A = "REQUEST_COOKIES|!REQUEST_COOKIES:/__utm/|REQUEST_COOKIES_NAMES|ARGS_NAMES|ARGS|XML:/*"
AH = "REQUEST_COOKIES|!REQUEST_COOKIES:/__utm/|REQUEST_COOKIES_NAMES|REQUEST_HEADERS:User-Agent|REQUEST_HEADERS:Referer|ARGS_NAMES|ARGS|XML:/*"
XT = "t:none,t:utf8toUnicode,t:urlDecodeUni,t:htmlEntityDecode,t:jsDecode,t:cssDecode,t:removeNulls"
ST = "t:none,t:urlDecodeUni"

# (file, gate id prefix, pl, id, targets, operator, transforms, msg, tag, score var, category var)
RULES = [
    # ---- 942 SQLi, PL2
    ("REQUEST-941-942-XSS-SQLI.conf", "942", 2, 942200, A,
     r"@rx (?i),.*?[)\da-f\"'`][\"'`](?:[\"'`].*?[\"'`]|(?:\r?\n)?\z|[^\"'`]+)|\Wselect.+\W*from|(?:alter|(?:(?:cre|trunc|upd)at|renam)e|d(?:e(?:lete|sc)|rop)|(?:inser|selec)t|load)[\s\x0b]*\([\s\x0b]*space[\s\x0b]*\(",
     "t:none,t:urlDecodeUni,t:removeCommentsChar", "Detects MySQL comment-/space-obfuscated injections and backtick termination", "attack-sqli", "critical", "sql_injection_score"),
    ("REQUEST-941-942-XSS-SQLI.conf", "942", 2, 942210, A,
     r"@rx (?i)(?:&&|\|\||and|between|div|like|n(?:and|ot)|(?:xx?)?or)[\s\x0b\(]+[0-9A-Z_a-z]+[\s\x0b]*?[!\+=]+[\s\x0b]*?[0-9]+",
     ST, "Detects chained SQL injection attempts 1/2", "attack-sqli", "critical", "sql_injection_score"),
    ("REQUEST-941-942-XSS-SQLI.conf", "942", 2, 942300, A,
     r"@rx (?i)\)[\s\x0b]*when[\s\x0b]+[0-9]+[\s\x0b]+then|[\"'`][\s\x0b]*(?:#|--|\{)|/\*![\s\x0b]?[0-9]+|\b(?:(?:binary|cha?r)[\s\x0b]*\(|(?:collate|into)[\s\x0b]+)",
     ST, "Detects MySQL comments, conditions and ch(a)r injections", "attack-sqli", "critical", "sql_injection_score"),
    ("REQUEST-941-942-XSS-SQLI.conf", "942", 2, 942310, A,
     r"@rx (?i)\([\s\x0b]*select[\s\x0b]*[0-9A-Z_a-z]+|\bcoalesce\b|order[\s\x0b]+by[\s\x0b]+if[0-9A-Z_a-z]*?[\s\x0b]*\(|[\"'`];*?[\s\x0b]*(?:having|select|union\b[\s\x0b]*(?:all|(?:distin|sele)ct))\b[\s\x0b]*[^\s\x0b]",
     ST, "Detects chained SQL injection attempts 2/2", "attack-sqli", "critical", "sql_injection_score"),
    ("REQUEST-941-942-XSS-SQLI.conf", "942", 2, 942340, A,
     r"@rx (?i)in[\s\x0b]*?\(+[\s\x0b]*?select|(?:(?:n?and|x?x?or|div|like|between)[\s\x0b]+|(?:\|\||&&)[\s\x0b]*)[\s\x0b\+]+[\"'`]|[\"'`]\|\|[\"'`]|[0-9][\s\x0b]*?(?:&&|\|\|)",
     ST, "Detects basic SQL authentication bypass attempts 3/3", "attack-sqli", "critical", "sql_injection_score"),
    ("REQUEST-941-942-XSS-SQLI.conf", "942", 2, 942360, A,
     r"@rx (?i)\b(?:(?:alter|(?:(?:cre|trunc|upd)at|renam)e|de(?:lete|sc)|(?:inser|selec)t|load)[\s\x0b]+(?:char|group_concat|load_file)\b[\s\x0b]*\(?|end[\s\x0b]*?\);)|[\s\x0b\(]load_file[\s\x0b]*?\(|[\"'`][\s\x0b]+regexp[^0-9A-Z_a-z]|[0-9A-Z_a-z]+[\s\x0b]*?\([\s\x0b]*\)[\s\x0b]*(?:from|into)\b",
     ST, "Detects concatenated basic SQL injection and SQLLFI attempts", "attack-sqli", "critical", "sql_injection_score"),
    ("REQUEST-941-942-XSS-SQLI.conf", "942", 2, 942370, A,
     r"@rx (?i)[\"'`](?:[\s\x0b]*?(?:\*.+(?:x?or|div|like|between|(?:an|i)d)[^0-9A-Z_a-z]*?[\"'`]|(?:x?or|div|like|between|and)[\s\x0b][^0-9]+[\-0-9A-Z_a-z]+.*?[0-9]))",
     ST, "Detects classic SQL injection probings 2/3", "attack-sqli", "critical", "sql_injection_score"),
    ("REQUEST-941-942-XSS-SQLI.conf", "942", 2, 942380, A,
     r"@rx (?i)\b(?:having\b(?:[\s\x0b]+(?:[0-9]{1,10}|'[^=]{1,10}')[\s\x0b]*?[<->]| ?(?:[0-9]{1,10} ?[<->]+|[\"'][^=]{1,10}[ \"'<-\?\[]+))|ex(?:ecute(?:\(|[\s\x0b]{1,5}[\$\.0-9A-Z_a-z]{1,5}[\s\x0b]{0,3})|ists[\s\x0b]*?\([\s\x0b]*?select\b)|(?:create[\s\x0b]+?table.{0,20}?|like[^0-9A-Z_a-z]*?char[^0-9A-Z_a-z]*?)\()",
     ST, "SQL Injection Attack", "attack-sqli", "critical", "sql_injection_score"),
    ("REQUEST-941-942-XSS-SQLI.conf", "942", 2, 942400, A,
     r"@rx (?i)\band\b(?:[\s\x0b]+(?:[0-9]{1,10}[\s\x0b]*?[<->]|'[^=]{1,10}')| ?(?:[0-9]{1,10}|[\"'][^=]{1,10}[\"']) ?[<->]+)",
     ST, "SQL Injection Attack", "attack-sqli", "critical", "sql_injection_score"),
    ("REQUEST-941-942-XSS-SQLI.conf", "942", 2, 942410, A,
     r"@rx (?i)\b(?:a(?:(?:b|co)s|dd(?:dat|tim)e|es_(?:de|en)crypt|s(?:in|cii(?:str)?)|tan2?|vg)|b(?:enchmark|i(?:n(?:_to_num)?|t_(?:and|count|length|x?or)))|c(?:har(?:acter)?_length|iel(?:ing)?|o(?:alesce|ercibility|llation|(?:mpres)?s|n(?:cat(?:_ws)?|nection_id|v(?:ert(?:_tz)?)?)|t)|r32|ur(?:(?:dat|tim)e|rent_(?:date|setting|time(?:stamp)?|user)))|d(?:a(?:t(?:abase(?:_to_xml)?|e(?:_(?:add|format|sub)|diff))|y(?:name|of(?:month|week|year)))|count|e(?:code|s_(?:de|en)crypt)|ump)|load_file|sleep|pg_sleep|benchmark|extractvalue|updatexml)[\s\x0b]*?\(",
     ST, "SQL Injection Attack: SQL function call", "attack-sqli", "critical", "sql_injection_score"),
    ("REQUEST-941-942-XSS-SQLI.conf", "942", 2, 942430, "ARGS_NAMES|ARGS|XML:/*",
     r"@rx ((?:[~!@#\$%\^&\*\(\)\-\+=\{\}\[\]\|:;\"'\xc2\xb4\x60<>][^~!@#\$%\^&\*\(\)\-\+=\{\}\[\]\|:;\"'\xc2\xb4\x60<>]*?){12})",
     ST, "Restricted SQL Character Anomaly Detection (args): # of special characters exceeded (12)", "attack-sqli", "warning", "sql_injection_score"),
    ("REQUEST-941-942-XSS-SQLI.conf", "942", 2, 942440, A,
     r"@rx /\*!?|\*/|[';]--|--(?:[\s\x0b]|[^\-]*?-)|[^&\-]#.*?[\s\x0b]|;?\x00",
     ST, "SQL Comment Sequence Detected", "attack-sqli", "critical", "sql_injection_score"),
    ("REQUEST-941-942-XSS-SQLI.conf", "942", 2, 942450, A,
     r"@rx (?i)\b0x[0-9a-f]{2,}", ST, "SQL Hex Encoding Identified", "attack-sqli", "critical", "sql_injection_score"),
    ("REQUEST-941-942-XSS-SQLI.conf", "942", 2, 942470, A,
     r"@rx (?i)autonomous_transaction|(?:current_use|n?varcha|tbcreato)r|db(?:a_users|ms_java)|open(?:owa_util|query|rowset)|s(?:p_(?:(?:addextendedpro|sqlexe)c|execute(?:sql)?|help|is_srvrolemember|makewebtask|oacreate|p(?:assword|repare)|replwritetovarbin)|ql_(?:longvarchar|variant))|utl_(?:file|http)|xp_(?:availablemedia|(?:cmdshel|servicecontro)l|dirtree|e(?:numdsn|xecresultset)|filelist|loginconfig|makecab|ntsec(?:_enumdomains)?|reg(?:addmultistring|delete(?:key|value)|enum(?:key|value)s|re(?:ad|movemultistring)|write)|terminate(?:_process)?)",
     ST, "SQL Injection Attack", "attack-sqli", "critical", "sql_injection_score"),
    ("REQUEST-941-942-XSS-SQLI.conf", "942", 2, 942480, "REQUEST_COOKIES|!REQUEST_COOKIES:/__utm/|REQUEST_COOKIES_NAMES|REQUEST_HEADERS|ARGS_NAMES|ARGS|XML:/*",
     r"@rx (?i)\b(?:(?:d(?:bms_[0-9A-Z_a-z]+\.|elete\b[^0-9A-Z_a-z]*?\bfrom)|(?:group\b.*?\bby\b.{1,100}?\bhav|overlay\b[^0-9A-Z_a-z]*?\(.*?\b[^0-9A-Z_a-z]*?plac)ing|in(?:ner\b[^0-9A-Z_a-z]*?\bjoin|sert\b[^0-9A-Z_a-z]*?\binto|to\b[^0-9A-Z_a-z]*?\b(?:dump|out)file)|load\b[^0-9A-Z_a-z]*?\bdata\b.*?\binfile|s(?:elect\b.{1,100}?\b(?:(?:.*?\bdump\b.*|(?:count|length)\b.{1,100}?)\bfrom|(?:data_typ|from\b.{1,100}?\bwher)e|instr|to(?:_(?:cha|numbe)r|p\b.{1,100}?\bfrom))|ys_context)|u(?:nion\b.{1,100}?\bselect|tl_inaddr))\b|print\b[^0-9A-Z_a-z]*?@@)|(?:collation[^0-9A-Z_a-z]*?\(a|@@version|;[^0-9A-Z_a-z]*?\b(?:drop|shutdown))\b|'(?:dbo|msdasql|s(?:a|qloledb))'",
     "t:none,t:urlDecodeUni,t:lowercase", "SQL Injection Attack", "attack-sqli", "critical", "sql_injection_score"),
    ("REQUEST-941-942-XSS-SQLI.conf", "942", 2, 942510, A,
     r"@rx (?:`(?:(?:[\w\s=_\-+{}()<@]){2,29}|(?:[A-Za-z0-9+/]{4})+(?:[A-Za-z0-9+/]{2}==|[A-Za-z0-9+/]{3}=)?)`)",
     ST, "SQLi bypass attempt by ticks or backticks detected", "attack-sqli", "critical", "sql_injection_score"),
    # ---- 942 SQLi, PL3
    ("REQUEST-941-942-XSS-SQLI.conf", "942", 3, 942251, A,
     r"@rx (?i)\W+\d*?\s*?\bhaving\b\s*?[^\s\-]", ST, "Detects HAVING injections", "attack-sqli", "critical", "sql_injection_score"),
    ("REQUEST-941-942-XSS-SQLI.conf", "942", 3, 942490, "ARGS_NAMES|ARGS|XML:/*",
     r"@rx [\"'`][\s\d]*?[^\w\s]\W*?\d\W*?.*?[\"'`\d]", ST, "Detects classic SQL injection probings 3/3", "attack-sqli", "critical", "sql_injection_score"),
    ("REQUEST-941-942-XSS-SQLI.conf", "942", 3, 942420, "REQUEST_COOKIES|!REQUEST_COOKIES:/__utm/|REQUEST_COOKIES_NAMES",
     r"@rx ((?:[~!@#\$%\^&\*\(\)\-\+=\{\}\[\]\|:;\"'\xc2\xb4\x60<>][^~!@#\$%\^&\*\(\)\-\+=\{\}\[\]\|:;\"'\xc2\xb4\x60<>]*?){8})",
     ST, "Restricted SQL Character Anomaly Detection (cookies): # of special characters exceeded (8)", "attack-sqli", "warning", "sql_injection_score"),
    # ---- 942 SQLi, PL4
    ("REQUEST-941-942-XSS-SQLI.conf", "942", 4, 942421, "REQUEST_COOKIES|!REQUEST_COOKIES:/__utm/|REQUEST_COOKIES_NAMES",
     r"@rx ((?:[~!@#\$%\^&\*\(\)\-\+=\{\}\[\]\|:;\"'\xc2\xb4\x60<>][^~!@#\$%\^&\*\(\)\-\+=\{\}\[\]\|:;\"'\xc2\xb4\x60<>]*?){3})",
     ST, "Restricted SQL Character Anomaly Detection (cookies): # of special characters exceeded (3)", "attack-sqli", "warning", "sql_injection_score"),
    ("REQUEST-941-942-XSS-SQLI.conf", "942", 4, 942460, "ARGS",
     r"@rx \W{4}", "t:none", "Meta-Character Anomaly Detection Alert - Repetitive Non-Word Characters", "attack-sqli", "warning", "sql_injection_score"),
    # ---- 941 XSS, PL2
    ("REQUEST-941-942-XSS-SQLI.conf", "941", 2, 941320, A,
     r"@rx (?i)<(?:a|abbr|acronym|address|applet|area|audioscope|b|base|basefront|bdo|bgsound|big|blackface|blink|blockquote|body|bq|br|button|caption|center|cite|code|col|colgroup|comment|dd|del|dfn|dir|div|dl|dt|em|embed|fieldset|fn|font|form|frame|frameset|h1|head|hr|html|i|iframe|ilayer|img|input|ins|isindex|kdb|keygen|label|layer|legend|li|limittext|link|listing|map|marquee|menu|meta|multicol|nobr|noembed|noframes|noscript|nosmartquotes|object|ol|optgroup|option|p|param|plaintext|pre|q|rt|ruby|s|samp|script|select|server|shadow|sidebar|small|spacer|span|strike|strong|style|sub|sup|table|tbody|td|textarea|tfoot|th|thead|title|tr|tt|u|ul|var|wbr|xml|xmp)\W",
     XT, "Possible XSS Attack Detected - HTML Tag Handler", "attack-xss", "critical", "xss_score"),
    ("REQUEST-941-942-XSS-SQLI.conf", "941", 2, 941330, A,
     r"@rx (?i)[\"'][\s\x0b]*(?:[^a-z0-9~_:' \x0b]|in).*?(?:(?:l|\x5cu006C)(?:o|\x5cu006F)(?:c|\x5cu0063)(?:a|\x5cu0061)(?:t|\x5cu0074)(?:i|\x5cu0069)(?:o|\x5cu006F)(?:n|\x5cu006E)|(?:n|\x5cu006E)(?:a|\x5cu0061)(?:m|\x5cu006D)(?:e|\x5cu0065)|(?:o|\x5cu006F)(?:n|\x5cu006E)(?:e|\x5cu0065)(?:r|\x5cu0072)(?:r|\x5cu0072)(?:o|\x5cu006F)(?:r|\x5cu0072)|(?:v|\x5cu0076)(?:a|\x5cu0061)(?:l|\x5cu006C)(?:u|\x5cu0075)(?:e|\x5cu0065)(?:O|\x5cu004F)(?:f|\x5cu0066)).*?=",
     XT, "IE XSS Filters - Attack Detected", "attack-xss", "critical", "xss_score"),
    ("REQUEST-941-942-XSS-SQLI.conf", "941", 2, 941340, A,
     r"@rx (?i)[\"\'][\s\x0b]*(?:[^a-z0-9~_:\' \x0b]|in).+?[\.].+?=", XT, "IE XSS Filters - Attack Detected", "attack-xss", "critical", "xss_score"),
    ("REQUEST-941-942-XSS-SQLI.conf", "941", 2, 941380, A,
     r"@rx \{\{.*?\}\}", "t:none", "AngularJS client side template injection detected", "attack-xss", "critical", "xss_score"),
    # ---- 941 XSS, PL3
    ("REQUEST-941-942-XSS-SQLI.conf", "941", 3, 941360, A,
     r"@rx ![!+ ]\[\]", XT, "JSFuck / Hieroglyphy obfuscation detected", "attack-xss", "critical", "xss_score"),
    # ---- 941 XSS, PL4 (the response-side rules of CRS are out of the path)
    ("REQUEST-941-942-XSS-SQLI.conf", "941", 4, 941400, A,
     r"@rx (?i)\[\s*\]\s*\[\s*(?:!\s*!\s*\[\s*\]|\+\s*\[\s*\])", XT, "XSS JavaScript function without parentheses", "attack-xss", "critical", "xss_score"),
    # ---- 920 protocol, PL2-PL4
    ("REQUEST-911-920-921-PROTOCOL.conf", "920", 2, 920230, "ARGS",
     r"@rx %[0-9a-fA-F]{2}", "t:none,t:urlDecodeUni", "Multiple URL Encoding Detected", "attack-protocol", "warning", None),
    ("REQUEST-911-920-921-PROTOCOL.conf", "920", 2, 920271, "REQUEST_URI|REQUEST_HEADERS|ARGS|ARGS_NAMES",
     "@validateByteRange 9,10,13,32-126,128-255", "t:none,t:urlDecodeUni", "Invalid character in request (non printable characters)", "attack-protocol", "critical", None),
    ("REQUEST-911-920-921-PROTOCOL.conf", "920", 2, 920320, "REQUEST_HEADERS_NAMES",
     r"@rx (?i)^(?:x-(?:forwarded|real|originating|remote)-(?:for|ip|addr)|client-ip)$", "t:none",
     "Forwarded-for header present (proxy chain)", "attack-protocol", "notice", None),
    ("REQUEST-911-920-921-PROTOCOL.conf", "920", 3, 920272, "REQUEST_URI|REQUEST_HEADERS|ARGS|ARGS_NAMES",
     "@validateByteRange 32-36,38-126", "t:none,t:urlDecodeUni", "Invalid character in request (outside of printable chars below ascii 127)", "attack-protocol", "critical", None),
    ("REQUEST-911-920-921-PROTOCOL.conf", "920", 3, 920300, "REQUEST_HEADERS:Accept",
     r"@rx ^$", "t:none", "Request Missing an Accept Header", "attack-protocol", "notice", None),
    ("REQUEST-911-920-921-PROTOCOL.conf", "920", 4, 920273, "ARGS|ARGS_NAMES|REQUEST_COOKIES|!REQUEST_COOKIES:/__utm/|REQUEST_COOKIES_NAMES",
     "@validateByteRange 38,44-46,48-58,61,65-90,95,97-122", "t:none,t:urlDecodeUni", "Invalid character in request (outside of very strict set)", "attack-protocol", "critical", None),
    ("REQUEST-911-920-921-PROTOCOL.conf", "920", 4, 920274, "REQUEST_HEADERS|!REQUEST_HEADERS:User-Agent|!REQUEST_HEADERS:Referer|!REQUEST_HEADERS:Cookie|!REQUEST_HEADERS:Sec-Fetch-User|!REQUEST_HEADERS:Sec-CH-UA-Mobile",
     "@validateByteRange 32,34,38,42-59,61,65-90,95,97-122", "t:none,t:urlDecodeUni", "Invalid character in request headers (outside of very strict set)", "attack-protocol", "critical", None),
    ("REQUEST-911-920-921-PROTOCOL.conf", "920", 4, 920460, "REQUEST_URI|REQUEST_HEADERS|ARGS|ARGS_NAMES",
     r"@rx (?:^|[^\x5c])\x5c[cdeghijklmpqwxyz123456789]", "t:none,t:htmlEntityDecode,t:lowercase", "Abnormal character escapes in request", "attack-protocol", "critical", None),
    # ---- 921 protocol attack, PL2-PL3
    ("REQUEST-911-920-921-PROTOCOL.conf", "921", 2, 921151, "ARGS_GET",
     r"@rx [\n\r]", "t:none,t:htmlEntityDecode", "HTTP Header Injection Attack via payload (CR/LF detected)", "attack-protocol", "critical", None),
    ("REQUEST-911-920-921-PROTOCOL.conf", "921", 3, 921230, "REQUEST_HEADERS:Range",
     r"@rx (?i)^(?:bytes=)?(?:[0-9]*-[0-9]*,){5,}", "t:none", "HTTP Range Header detected", "attack-protocol", "critical", None),
    # ---- 932 RCE, PL2-PL3
    ("REQUEST-930-934-ATTACKS.conf", "932", 2, 932200, "REQUEST_COOKIES|!REQUEST_COOKIES:/__utm/|REQUEST_COOKIES_NAMES|REQUEST_HEADERS:Referer|REQUEST_HEADERS:User-Agent|ARGS_NAMES|ARGS|XML:/*",
     r"@rx ['\*\?\x5c`][^\n/]+/|/[^/]+?['\*\?\x5c`]|\$[!#\$\(\*\-0-9\?-\[_a-\{]", "t:none,t:lowercase,t:urlDecodeUni",
     "RCE Bypass Technique", "attack-rce", "critical", "rce_score"),
    ("REQUEST-930-934-ATTACKS.conf", "932", 2, 932230, A,
     r"@rx (?i)(?:^|=|[;&\|\(\)\{\}`]|\$\(|\$\(\()[\s\x0b]*(?:[\"'\x5c]*(?:l[\"'\x5c]*s|c[\"'\x5c]*a[\"'\x5c]*t|w[\"'\x5c]*g[\"'\x5c]*e[\"'\x5c]*t|c[\"'\x5c]*u[\"'\x5c]*r[\"'\x5c]*l|n[\"'\x5c]*c|i[\"'\x5c]*d|u[\"'\x5c]*n[\"'\x5c]*a[\"'\x5c]*m[\"'\x5c]*e|w[\"'\x5c]*h[\"'\x5c]*o[\"'\x5c]*a[\"'\x5c]*m[\"'\x5c]*i))(?:[\s\x0b<>&\|\)]|$)",
     "t:none,t:cmdLine", "Remote Command Execution: Unix Command Injection", "attack-rce", "critical", "rce_score"),
    ("REQUEST-930-934-ATTACKS.conf", "932", 3, 932190, A,
     r"@rx /(?:[?*]+[a-z/]+|[a-z/]+[?*]+)", "t:none,t:cmdLine,t:normalizePath", "Remote Command Execution: Wildcard bypass technique attempt", "attack-rce", "critical", "rce_score"),
    # ---- 933 PHP, PL2-PL3
    ("REQUEST-930-934-ATTACKS.conf", "933", 2, 933151, A,
     r"@rx (?i)\b(?:a(?:rray_(?:map|walk)|ssert)|call_user_func(?:_array)?|create_function|e(?:scapeshellcmd|x(?:ec|tract))|f(?:ile_(?:get|put)_contents|open|write)|p(?:assthru|cntl_exec|open|roc_open|reg_replace)|s(?:hell_exec|ystem)|unserialize)[\s\x0b]*\(",
     "t:none,t:lowercase", "PHP Injection Attack: Medium-Risk PHP Function Name Found", "attack-php", "critical", "php_injection_score"),
    ("REQUEST-930-934-ATTACKS.conf", "933", 3, 933161, A,
     r"@rx (?i)\b(?:a(?:bs|cos|sin|tan)|b(?:ase64_(?:de|en)code|in2hex)|c(?:eil|hr|os|rc32|url_exec)|d(?:ate|ecbin|echex|ir)|f(?:loor|mod|putcsv)|g(?:et(?:env|cwd)|lob)|h(?:ex2bin|tmlspecialchars)|i(?:mplode|ni_set|s_(?:dir|file))|l(?:ink|og)|m(?:ail|d5|kdir)|o(?:b_start|rd)|p(?:hpinfo|ow|rint_r)|r(?:ename|mdir|ound)|s(?:ha1|in|leep|printf|qrt|trrev|ubstr)|t(?:an|ouch)|u(?:mask|nlink|rldecode)|var_dump)(?:[\s\x0b]|/\*.*\*/|#.*|//.*)*\(.*\)",
     "t:none,t:lowercase", "PHP Injection Attack: Low-Value PHP Function Call Detected", "attack-php", "critical", "php_injection_score"),
    # ---- 934 generic, PL2
    ("REQUEST-930-934-ATTACKS.conf", "934", 2, 934101, A,
     r"@rx (?i)\b(?:child_process|process\.(?:binding|dlopen|env|kill|mainModule)|require\s*\(\s*['\"](?:fs|net|vm|http)['\"]|this\.constructor|__proto__|constructor\s*\[)",
     "t:none,t:urlDecodeUni,t:jsDecode,t:base64Decode", "Node.js Injection Attack 2/2", "attack-injection-generic", "critical", None),
]

SCORES = {"critical": "critical_anomaly_score", "warning": "warning_anomaly_score",
          "notice": "notice_anomaly_score", "error": "error_anomaly_score"}


def rule_text(pl, rid, targets, op, tr, msg, tag, sev, cat):
    lines = ['SecRule %s "%s" \\' % (targets, op),
             '    "id:%d,\\' % rid, "    phase:2,\\", "    block,\\", "    capture,\\", "    %s,\\" % tr,
             "    msg:'%s',\\" % msg.replace("'", ""),
             "    logdata:'Matched Data: %{TX.0} found within %{MATCHED_VAR_NAME}: %{MATCHED_VAR}',\\",
             "    tag:'%s',\\" % tag, "    tag:'paranoia-level/%d',\\" % pl, "    ver:'OWASP_CRS/4.23.0',\\",
             "    severity:'%s',\\" % sev.upper()]
    sets = []
    if cat:
        sets.append("    setvar:'tx.%s=+%%{tx.%s}'" % (cat, SCORES[sev]))
    sets.append("    setvar:'tx.inbound_anomaly_score_pl%d=+%%{tx.%s}'" % (pl, SCORES[sev]))
    lines += [s + ",\\" for s in sets[:-1]] + [sets[-1] + '"']
    return "\n".join(lines) + "\n"


def main():
    added = 0
    for fname in sorted({r[0] for r in RULES}):
        path = os.path.join(CRS, fname)
        text = open(path).read()
        for (f, sec, pl, rid, targets, op, tr, msg, tag, sev, cat) in RULES:
            if f != fname or ("id:%d," % rid) in text:
                continue
            # insert before the gate that closes level `pl` (the "@lt pl+1" pair), or the END marker for PL4
            if pl < 4:
                m = re.search(r'SecRule TX:DETECTION_PARANOIA_LEVEL "@lt %d" "id:%s0%d' % (pl + 1, sec, 11 + 2 * pl), text)
            else:
                m = None
                for mm in re.finditer(r'SecMarker "END-REQUEST-%s-[A-Z-]+"' % sec, text):
                    m = mm
                    break
            if m is None:
                raise SystemExit("no gate for %s PL%d in %s" % (sec, pl, fname))
            text = text[:m.start()] + rule_text(pl, rid, targets, op, tr, msg, tag, sev, cat) + "\n" + text[m.start():]
            added += 1
        open(path, "w").write(text)
    print("added", added, "rules")


if __name__ == "__main__":
    main()
