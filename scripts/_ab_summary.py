import json
import sys
for l in open(sys.argv[1]):
    if l.startswith(('room', 'seabed')):
        name, rest = l.split(' ', 1)
        d = json.loads(rest.split('} ')[0] + '}')
        keys = [k for k in d if k.startswith('normals_lists') or k.startswith('normals_chain')] + ['normals']
        print(name, ' '.join('%s %.3f' % (k.replace('normals_', ''), d[k]) for k in keys))
    elif l.startswith(('==', 'bench')):
        print(l.rstrip())
