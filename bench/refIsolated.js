/**
 * Start the process that runs the reference's pages (bench/refWorker.cjs)
 * and talk to it in JSON lines (ADR 014).
 *
 * The process is denied network and writes with what this container has
 * (util-linux): `unshare --net --mount` gives it an empty network namespace
 * and a mount namespace whose mounts are remounted read-only (the root must
 * be; /proc and the like where they allow it); `prlimit --fsize=0` stops
 * file writes on any mount that stays writable;
 * `setpriv` drops every capability (so it cannot remount, and cannot read
 * past the owner-only /root) and sets no_new_privs. Node starts with
 * --disallow-code-generation-from-strings and an environment of PATH alone.
 * The worker's source goes on its command line and everything else —
 * React, the DOM stand-in, the reference's transpiled modules, the cluster —
 * through its stdin: it opens no file. Without these tools (an unprivileged
 * container) the start fails and the comparison does not run.
 */
import { spawn } from 'child_process';
import fs from 'fs';
import path from 'path';
import { fileURLToPath } from 'url';
import { bundle } from '../tools/bundle.js';
import { referenceModules } from './referenceRender.js';

const HERE = path.dirname(fileURLToPath(import.meta.url));

/**
 * The shell step inside the new namespaces: the root read-only (required),
 * every other mount read-only where it can be, then no file size, no
 * capabilities, the worker.
 */
const LOCKDOWN = 'mount -o remount,bind,ro / && for m in $(awk \'{print $2}\' /proc/self/mounts); do ' +
  'mount -o remount,bind,ro "$m" 2>/dev/null; done; exec prlimit --fsize=0 -- setpriv --bounding-set=-all --inh-caps=-all ' +
  '--no-new-privs -- "$0" --disallow-code-generation-from-strings -e "$1"';

/** The command line of the isolated worker: [file, args]. */
export function workerCommand() {
  const src = fs.readFileSync(path.join(HERE, 'refWorker.cjs'), 'utf8');
  const boot = src + "\nprocess.on('SIGXFSZ', function () {});\nserve(require('vm'), process, require);\n";
  return ['unshare', ['--net', '--mount', '--propagation', 'private', '--', 'sh', '-c', LOCKDOWN, process.execPath, boot]];
}

/** How long one call may take before the worker is killed (ms): building the realm, and anything after it. */
export const INIT_TIMEOUT_MS = 120000;
export const CALL_TIMEOUT_MS = 60000;

/**
 * Start the worker → {call(cmd, fields, timeoutMs): Promise, close()}. A start
 * that fails (no unshare / setpriv, or no permission for them) rejects the
 * first call with the process's stderr. A call not answered in time (a
 * reference render that never returns, say) kills the worker and rejects
 * every call waiting and every later one: the realm's own timeout covers its
 * module code only, not the renders React runs afterwards.
 */
export function startWorker() {
  const cmd = workerCommand();
  const child = spawn(cmd[0], cmd[1], { stdio: ['pipe', 'pipe', 'pipe'], env: { PATH: process.env.PATH || '/usr/bin:/bin' }, cwd: '/' });
  const waiting = new Map();
  let next = 0;
  let buf = '';
  let err = '';
  let dead = null;
  child.stdout.setEncoding('utf8');
  child.stdout.on('data', function (chunk) {
    buf += chunk;
    let nl;
    while ((nl = buf.indexOf('\n')) >= 0) {
      const line = buf.slice(0, nl);
      buf = buf.slice(nl + 1);
      const m = JSON.parse(line);
      const w = waiting.get(m.id);
      if (!w) continue;
      waiting.delete(m.id);
      clearTimeout(w.timer);
      if (m.ok) w.resolve(m.result);
      else w.reject(new Error('reference worker: ' + m.error));
    }
  });
  child.stdin.on('error', function () {}); // a killed worker's pipe: the call is already rejected
  child.stderr.setEncoding('utf8');
  child.stderr.on('data', function (c) { err = (err + c).slice(-4000); });
  function fail(why) {
    if (!dead) dead = new Error('reference worker ' + why + (err ? ': ' + err.trim() : ''));
    waiting.forEach(function (w) { clearTimeout(w.timer); w.reject(dead); });
    waiting.clear();
  }
  child.on('error', function (e) { fail('did not start (' + e.message + ')'); });
  child.on('exit', function (code, sig) { fail('exited (' + (sig || code) + ')'); });
  return {
    call: function (cmd, fields, timeoutMs) {
      if (dead) return Promise.reject(dead);
      const id = ++next;
      const limit = timeoutMs || (cmd === 'init' ? INIT_TIMEOUT_MS : CALL_TIMEOUT_MS);
      return new Promise(function (resolve, reject) {
        const timer = setTimeout(function () {
          fail('timed out after ' + limit + ' ms on ' + cmd);
          child.kill('SIGKILL');
        }, limit);
        waiting.set(id, { resolve: resolve, reject: reject, timer: timer });
        child.stdin.write(JSON.stringify(Object.assign({ id: id, cmd: cmd }, fields || {})) + '\n');
      });
    },
    close: function () {
      child.stdin.end();
      return new Promise(function (resolve) {
        if (dead) resolve();
        else child.on('exit', function () { resolve(); });
      });
    },
  };
}

/** The realm's build message: the harness bundle, React's UMD sources, the reference's modules. */
export function realmInit(referenceDir, umdDir) {
  const ref = referenceModules(referenceDir);
  return {
    harness: bundle(path.join(HERE, 'refHarness.js')).code,
    react: fs.readFileSync(path.join(umdDir, 'react@18.3.1.min.js'), 'utf8'),
    reactDom: fs.readFileSync(path.join(umdDir, 'react-dom@18.3.1.min.js'), 'utf8'),
    modules: ref.modules,
    resolve: ref.resolve,
    pages: ref.pages,
  };
}

/** The reference's pages, ready to mount in the isolated worker: startWorker() after its `init`. */
export async function referenceWorker(referenceDir, umdDir) {
  const w = startWorker();
  try {
    await w.call('init', realmInit(referenceDir, umdDir));
  } catch (e) {
    await w.close();
    throw e;
  }
  return w;
}
